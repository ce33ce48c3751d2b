// tests/hip/libm_probe.hip -- TEST-ONLY check that the device build of libm_f32.h (the kernel's sky
// UV atan2f / asinf) returns the host glibc's bits. Built and run by tests/test_gpu_probes.py.
//   asinf:         every float in [-1, 1]
//   atan2f(y, 1):  every finite y (the atanf core)
//   atan2f(y, x):  random pairs -- unit directions as WorldToSkyUV sees them, plus random bit patterns
// The device evaluates chunks of 2^26 inputs; 16 host threads compare against glibc.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "libm_f32.h"
#include "libm_f32_x2.h"

namespace {

constexpr uint64_t kChunk = 1ull << 26;

__host__ __device__ inline uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline float bits_to_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline uint32_t float_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
// Any NaN matches any NaN -- except the pair probes' "special element" marker, which must match exactly.
inline bool same(float a, float b) {
    if (float_bits(a) == 0x7fc0deadu || float_bits(b) == 0x7fc0deadu) return float_bits(a) == float_bits(b);
    return float_bits(a) == float_bits(b) || (a != a && b != b);
}

// Pair i of the random atan2f set (host and device agree on it).
__host__ __device__ inline void pair(uint64_t seed, uint64_t i, float& y, float& x) {
    const uint64_t h = mix(seed ^ (i * 0x100000001B3ull));
    const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
    if (i & 1) {  // a direction: components in [-1, 1], including near-zero and near-pole magnitudes
        const float a = (float)(lo >> 8) * 0x1p-23f - 1.0f;
        const float b = (float)(hi >> 8) * 0x1p-23f - 1.0f;
        const int sh = (int)((h >> 20) & 31);
        y = (i & 2) ? a * __builtin_ldexpf(1.0f, -sh) : a;
        x = (i & 4) ? b * __builtin_ldexpf(1.0f, -sh) : b;
    } else {
        y = __builtin_bit_cast(float, lo);
        x = __builtin_bit_cast(float, hi);
    }
}

__global__ void k_unary(int which, uint32_t base, uint64_t n, float* out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = __uint_as_float(base + (uint32_t)i);
    out[i] = which == 0 ? pbr_asinf(v) : pbr_atan2f(v, 1.0f);
}

__global__ void k_pairs(uint64_t seed, uint64_t first, uint64_t n, float* out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float y, x;
    pair(seed, first + i, y, x);
    out[i] = pbr_atan2f(y, x);
}

__constant__ pbr_atan_seg k_atan_tab[5] = PBR_ATAN_SEG_TABLE_INIT;

// The pair forms (libm_f32_x2.h): work-item i evaluates inputs 2i and 2i + 1 together; a special element (the
// caller's scalar fallback) is written as a NaN with payload 0x7fc0dead so the host can tell it apart.
__global__ void k_unary_x2(int which, uint32_t base, uint64_t n, float* out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (2 * i >= n) return;
    const pbr_lv2 v = {__uint_as_float(base + (uint32_t)(2 * i)), __uint_as_float(base + (uint32_t)(2 * i + 1))};
    int sp[2];
    const pbr_lv2 r = which == 0 ? pbr_asinf_x2(v, sp) : pbr_atan2f_x2(v, (pbr_lv2)(1.0f), sp, k_atan_tab);
    out[2 * i] = sp[0] ? __uint_as_float(0x7fc0deadu) : r.x;
    if (2 * i + 1 < n) out[2 * i + 1] = sp[1] ? __uint_as_float(0x7fc0deadu) : r.y;
}

__global__ void k_pairs_x2(uint64_t seed, uint64_t first, uint64_t n, float* out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (2 * i >= n) return;
    float y0, x0, y1, x1;
    pair(seed, first + 2 * i, y0, x0);
    pair(seed, first + 2 * i + 1, y1, x1);
    int sp[2];
    const pbr_lv2 r = pbr_atan2f_x2((pbr_lv2){y0, y1}, (pbr_lv2){x0, x1}, sp, k_atan_tab);
    out[2 * i] = sp[0] ? __uint_as_float(0x7fc0deadu) : r.x;
    if (2 * i + 1 < n) out[2 * i + 1] = sp[1] ? __uint_as_float(0x7fc0deadu) : r.y;
}

// The inputs the pair forms must hand to the scalar functions.
inline bool atan2_special(float y, float x) {
    auto in = [](float v) { const float a = std::fabs(v); return a == 0.0f || (a >= 0x1p-40f && a <= 0x1p40f); };
    return !(in(y) && in(x));
}

template <class F>
uint64_t compare_parallel(uint64_t n, const float* got, F expected, uint64_t* first_bad_index) {
    const int T = 16;
    std::vector<std::thread> th;
    std::atomic<uint64_t> bad{0};
    std::atomic<uint64_t> first{~0ull};
    for (int t = 0; t < T; ++t) {
        th.emplace_back([&, t] {
            uint64_t nb = 0, fb = ~0ull;
            for (uint64_t i = n * t / T; i < n * (t + 1) / T; ++i)
                if (!same(got[i], expected(i))) {
                    ++nb;
                    if (fb == ~0ull) fb = i;
                }
            bad += nb;
            uint64_t cur = first.load();
            while (fb < cur && !first.compare_exchange_weak(cur, fb)) {}
        });
    }
    for (auto& x : th) x.join();
    *first_bad_index = first.load();
    return bad.load();
}

}  // namespace

// which: 0 = asinf, 1 = atan2f(y, 1). Sweeps bit patterns [lo, hi] inclusive. Returns mismatches,
// or -1 on a HIP error; *first_bad = first mismatching bit pattern (0xffffffff if none).
extern "C" long long probe_unary(int which, uint32_t lo, uint32_t hi, uint32_t* first_bad) {
    float *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, kChunk * 4) != hipSuccess || hipHostMalloc(&h, kChunk * 4) != hipSuccess) return -1;
    long long bad = 0;
    *first_bad = 0xffffffffu;
    for (uint64_t base = lo; base <= hi; base += kChunk) {
        const uint64_t n = std::min<uint64_t>(kChunk, (uint64_t)hi - base + 1);
        hipLaunchKernelGGL(k_unary, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, which, (uint32_t)base, n, d);
        if (hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        uint64_t fi;
        const uint64_t b = compare_parallel(n, h, [&](uint64_t i) {
            const float v = bits_to_float((uint32_t)(base + i));
            return which == 0 ? asinf(v) : atan2f(v, 1.0f);
        }, &fi);
        if (b && *first_bad == 0xffffffffu) *first_bad = (uint32_t)(base + fi);
        bad += (long long)b;
    }
    hipFree(d);
    hipHostFree(h);
    return bad;
}

// n random atan2f pairs (see pair()). Returns mismatches or -1; *bad_y / *bad_x = first mismatch.
extern "C" long long probe_atan2_pairs(uint64_t seed, uint64_t n_total, float* bad_y, float* bad_x) {
    float *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, kChunk * 4) != hipSuccess || hipHostMalloc(&h, kChunk * 4) != hipSuccess) return -1;
    long long bad = 0;
    for (uint64_t first = 0; first < n_total; first += kChunk) {
        const uint64_t n = std::min<uint64_t>(kChunk, n_total - first);
        hipLaunchKernelGGL(k_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, seed, first, n, d);
        if (hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        uint64_t fi;
        const uint64_t b = compare_parallel(n, h, [&](uint64_t i) {
            float y, x;
            pair(seed, first + i, y, x);
            return atan2f(y, x);
        }, &fi);
        if (b && bad == 0) pair(seed, first + fi, *bad_y, *bad_x);
        bad += (long long)b;
    }
    hipFree(d);
    hipHostFree(h);
    return bad;
}

// The pair forms, checked like the scalar ones: `which` 0 = pbr_asinf_x2, 1 = pbr_atan2f_x2(y, 1) over the bit
// patterns [lo, hi]; an element they flag special must be exactly one the scalar function is needed for, every other
// element must carry glibc's bits. Returns mismatches (either kind) or -1; *first_bad as probe_unary.
extern "C" long long probe_unary_x2(int which, uint32_t lo, uint32_t hi, uint32_t* first_bad) {
    float *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, kChunk * 4) != hipSuccess || hipHostMalloc(&h, kChunk * 4) != hipSuccess) return -1;
    long long bad = 0;
    *first_bad = 0xffffffffu;
    for (uint64_t base = lo; base <= hi; base += kChunk) {
        const uint64_t n = std::min<uint64_t>(kChunk, (uint64_t)hi - base + 1);
        hipLaunchKernelGGL(k_unary_x2, dim3((unsigned)((n / 2 + 256) / 256)), dim3(256), 0, 0, which, (uint32_t)base, n, d);
        if (hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        uint64_t fi;
        const uint64_t b = compare_parallel(n, h, [&](uint64_t i) -> float {
            const float v = bits_to_float((uint32_t)(base + i));
            const bool special = which == 0 ? (std::fabs(v) > 1.0f || v != v) : atan2_special(v, 1.0f);
            if (special) return __builtin_bit_cast(float, 0x7fc0deadu);
            return which == 0 ? asinf(v) : atan2f(v, 1.0f);
        }, &fi);
        if (b && *first_bad == 0xffffffffu) *first_bad = (uint32_t)(base + fi);
        bad += (long long)b;
    }
    hipFree(d);
    hipHostFree(h);
    return bad;
}

extern "C" long long probe_atan2_pairs_x2(uint64_t seed, uint64_t n_total, float* bad_y, float* bad_x) {
    float *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, kChunk * 4) != hipSuccess || hipHostMalloc(&h, kChunk * 4) != hipSuccess) return -1;
    long long bad = 0;
    for (uint64_t first = 0; first < n_total; first += kChunk) {
        const uint64_t n = std::min<uint64_t>(kChunk, n_total - first);
        hipLaunchKernelGGL(k_pairs_x2, dim3((unsigned)((n / 2 + 256) / 256)), dim3(256), 0, 0, seed, first, n, d);
        if (hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        uint64_t fi;
        const uint64_t b = compare_parallel(n, h, [&](uint64_t i) -> float {
            float y, x;
            pair(seed, first + i, y, x);
            if (atan2_special(y, x)) return __builtin_bit_cast(float, 0x7fc0deadu);
            return atan2f(y, x);
        }, &fi);
        if (b && bad == 0) pair(seed, first + fi, *bad_y, *bad_x);
        bad += (long long)b;
    }
    hipFree(d);
    hipHostFree(h);
    return bad;
}
