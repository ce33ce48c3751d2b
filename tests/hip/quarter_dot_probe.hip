// tests/hip/quarter_dot_probe.hip -- TEST-ONLY probe of the faithful loop's rescaled invariants
// (pbr_device_math_x2.h faithful_scale / brdf_faithful_x2<LEAN, true>). Built and run by
// tests/test_gpu_probes.py with the product's fp flags.
//
// Claim under test: inside the fast window (normal components 0 or in [2^-20, 16]; H and L components 0
// or >= 2^-88), dot3(N/4, H) is exactly dot3(N, H) / 4, so
//   * lean waves (|N|^2 <= 1 + 2^-20, |H| <= 1 + 2^-21): the clamp bit of the dot's last add gives
//     max(N.H, 0) / 4 bit for bit;
//   * every wave: max(dot3(N/4, H), 0) == max(N.H, 0) / 4;
//   * the GGX denominator inner = n_dot_h^2 (a^2 - 1) + 1 from the scaled pair (N.H / 4, 16 (a^2 - 1)) has
//     the reference's bits;
//   * faithful_unscale restores every rescaled invariant bit for bit.
// Pairs mix random directions with H close to N (N.H near 1, where the GGX denominator cancels) and
// components forced to 0 or to the window's small magnitudes.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "pbr_device_math_x2.h"

using namespace pbr;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float unit_f(uint64_t h) { return (float)(h >> 40) * 0x1p-24f * 2.0f - 1.0f; }  // [-1, 1)
// 2^-e with e uniform in [elo, ehi], random significand and sign.
__device__ __forceinline__ float small_f(uint64_t h, int elo, int ehi) {
    const int e = elo + (int)((h >> 32) % (uint64_t)(ehi - elo + 1));
    const float m = __uint_as_float(((uint32_t)(127 - e) << 23) | (uint32_t)(h & 0x7FFFFF));
    return (h >> 63) ? -m : m;
}
__device__ __forceinline__ f3 normalized(f3 v) {
    const float s = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return mk3(v.x / s, v.y / s, v.z / s);
}

struct Sample {
    f3 n, h;
    float a2m1, omk, nv4;
};

__device__ Sample make_sample(uint64_t seed, int lean) {
    uint64_t s = mix(seed);
    Sample o;
    if (lean) {
        o.n = normalized(mk3(unit_f(s), unit_f(mix(s + 1)), unit_f(mix(s + 2))));
    } else {  // magnitudes across the window [2^-20, 16]
        o.n = mk3(small_f(mix(s + 1), -4, 20), small_f(mix(s + 2), -4, 20), small_f(mix(s + 3), -4, 20));
    }
    for (int c = 0; c < 3; ++c) {  // force some normal components to 0 or to the window's lower end
        const uint64_t r = mix(s + 10 + c);
        float& v = c == 0 ? o.n.x : (c == 1 ? o.n.y : o.n.z);
        if ((r & 15) == 0) v = 0.0f;
        else if ((r & 15) == 1) v = small_f(r, 10, 20);
    }
    const uint64_t kind = mix(s + 20) & 3;
    if (kind == 0) {  // H close to N: N.H near 1 (the ill-conditioned GGX spot)
        const float eps = small_f(mix(s + 21), 4, 24);
        o.h = normalized(mk3(o.n.x + eps * unit_f(mix(s + 22)), o.n.y + eps * unit_f(mix(s + 23)),
                             o.n.z + eps * unit_f(mix(s + 24))));
    } else {
        o.h = normalized(mk3(unit_f(mix(s + 25)), unit_f(mix(s + 26)), unit_f(mix(s + 27))));
    }
    for (int c = 0; c < 3; ++c) {  // H components 0 or as small as the window admits (2^-88)
        const uint64_t r = mix(s + 30 + c);
        float& v = c == 0 ? o.h.x : (c == 1 ? o.h.y : o.h.z);
        if ((r & 15) == 0) v = 0.0f;
        else if ((r & 15) == 1) v = small_f(r, 20, 88);
    }
    // Invariants as make_invariants forms them (roughness in [0, 1]; N.V 0 or >= 2^-100).
    const float rough = (float)(mix(s + 40) >> 40) * 0x1p-24f;
    const float r = fmaxf(rough, 0.05f), a = r * r;
    o.a2m1 = a * a - 1.0f;
    const float rr = rough + 1.0f;
    o.omk = 1.0f - (rr * rr) * 0.125f;
    const uint64_t nvr = mix(s + 41);
    o.nv4 = (nvr & 7) == 0 ? 0.0f : 4.0f * ((nvr & 7) == 1 ? small_f(nvr, 60, 100) : (float)(nvr >> 40) * 0x1p-24f);
    return o;
}

__device__ __forceinline__ bool same(float a, float b) { return __float_as_uint(a) == __float_as_uint(b); }

// bad[0]: dot mismatches, bad[1]: GGX inner mismatches, bad[2]: unscale mismatches; bad[3] (control):
// lanes with N.H > 1, where a plain saturate of the unscaled dot would have clamped the reference's value.
__global__ void quarter_dots(uint64_t seed, int iters, int lean, unsigned long long* bad) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned int nd = 0, ni = 0, nu = 0, nover = 0;
    for (int i = 0; i < iters; ++i) {
        const Sample a = make_sample(seed ^ (t * 0x100000001B3ull + 2 * (uint64_t)i), lean);
        const Sample b = make_sample(seed ^ (t * 0x100000001B3ull + 2 * (uint64_t)i + 1), lean);
        PixelInvariants2 q{};
        q.n = f3x2{v2{a.n.x, b.n.x}, v2{a.n.y, b.n.y}, v2{a.n.z, b.n.z}};
        q.a_sqr_minus_1 = v2{a.a2m1, b.a2m1};
        q.one_minus_k = v2{a.omk, b.omk};
        q.four_n_dot_v = v2{a.nv4, b.nv4};
        const f3x2 h = f3x2{v2{a.h.x, b.h.x}, v2{a.h.y, b.h.y}, v2{a.h.z, b.h.z}};
        PixelInvariants2 qs = q;
        faithful_scale(qs);
        const v2 ref = vmax(dot3(q.n, h), splat(0.0f));
        const v2 got = lean ? dot3_sat(qs.n, h) : vmax(dot3(qs.n, h), splat(0.0f));
        const v2 ref_inner = (ref * ref) * q.a_sqr_minus_1 + 1.0f;
        const v2 got_inner = (got * got) * qs.a_sqr_minus_1 + 1.0f;
        nd += !same(got.x, ref.x * 0.25f) + !same(got.y, ref.y * 0.25f);
        nover += (ref.x > 1.0f) + (ref.y > 1.0f);
        ni += !same(got_inner.x, ref_inner.x) + !same(got_inner.y, ref_inner.y);
        PixelInvariants2 qu = qs;
        faithful_unscale(qu);
        nu += !same(qu.n.x.x, q.n.x.x) + !same(qu.n.y.x, q.n.y.x) + !same(qu.n.z.x, q.n.z.x) +
              !same(qu.n.x.y, q.n.x.y) + !same(qu.n.y.y, q.n.y.y) + !same(qu.n.z.y, q.n.z.y) +
              !same(qu.a_sqr_minus_1.x, q.a_sqr_minus_1.x) + !same(qu.a_sqr_minus_1.y, q.a_sqr_minus_1.y) +
              !same(qu.one_minus_k.x, q.one_minus_k.x) + !same(qu.one_minus_k.y, q.one_minus_k.y) +
              !same(qu.four_n_dot_v.x, q.four_n_dot_v.x) + !same(qu.four_n_dot_v.y, q.four_n_dot_v.y);
    }
    if (nd) atomicAdd(&bad[0], (unsigned long long)nd);
    if (ni) atomicAdd(&bad[1], (unsigned long long)ni);
    if (nu) atomicAdd(&bad[2], (unsigned long long)nu);
    if (nover) atomicAdd(&bad[3], (unsigned long long)nover);
}

extern "C" int probe_quarter_dots(unsigned long long seed, int blocks, int iters, int lean, unsigned long long* bad) {
    unsigned long long* d_bad;
    if (blocks <= 0 || blocks > 65536 || iters <= 0) return -3;
    if (hipMalloc(&d_bad, 4 * 8) != hipSuccess) return -1;
    (void)hipMemset(d_bad, 0, 4 * 8);
    hipLaunchKernelGGL(quarter_dots, dim3(blocks), dim3(256), 0, 0, (uint64_t)seed, iters, lean, d_bad);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(bad, d_bad, 4 * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    return 0;
}
