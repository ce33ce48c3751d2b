// tests/hip/seed_div_probe.hip -- TEST-ONLY probe (gfx950): can the reciprocal that a normalize divides by come from
// the rsq seed its square root already computed, instead of a v_rcp?
//
// The kernels compute s = sqrt_nr(t) = RN(sqrt(t)) from y = rsq(t) and then 1/s as recip_nr(s) (v_rcp + one Newton
// step: RN(1/s) in the window) to divide by it with the Markstein step div_nr(a, s, r) = RN(a / s). The candidate
// reciprocal is r' = fma(fma(-s, y, 1), y, y), one Newton step from the seed y. It differs from RN(1/s) at one t per
// binade pair (s with an all-ones significand; DESIGN.md, "Tried and dropped"). What matters for a normalize is the
// quotient, not r': sweep 1 lists every t in the window whose r' != RN(1/s); sweep 2 divides every a with
// |a| <= s (a unit vector's components: |a / s| <= 1) and exponent down to 2^-40 below s's by that s with r' and
// compares the Markstein quotient with IEEE a / s (this file is built with -fhip-fp32-correctly-rounded-divide-sqrt).
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ float seed_sqrt(float t, float& y) {
    y = __builtin_amdgcn_rsqf(t);
    const float s0 = t * y;
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, t), 0.5f * y, s0);
}
__device__ __forceinline__ float seed_recip(float s, float y) { return __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y); }
__device__ __forceinline__ float rcp_recip(float s) {
    const float r0 = __builtin_amdgcn_rcpf(s);
    return __builtin_fmaf(__builtin_fmaf(-s, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ float markstein(float a, float s, float r) {
    const float q = a * r;
    const float e = __builtin_fmaf(s, q, -a);
    return __builtin_fmaf(-e, r, q);
}

// Sweep 1: every t with exponent in [emin, emax]; counts sqrt_nr != sqrtf, recip_nr != 1/s (controls, expect 0) and
// r' != 1/s, and lists the t of the last kind (at most `cap`).
__global__ void seed_sweep(int emin, int emax, unsigned long long* counts, uint32_t* list, int cap) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    unsigned int bad_sqrt = 0, bad_rcp = 0, bad_seed = 0;
    for (int e = emin; e <= emax; ++e) {
        const uint32_t bits = ((uint32_t)(e + 127) << 23) | m;
        const float t = __uint_as_float(bits);
        float y;
        const float s = seed_sqrt(t, y);
        const float exact = 1.0f / s;
        bad_sqrt += __float_as_uint(s) != __float_as_uint(sqrtf(t));
        bad_rcp += __float_as_uint(rcp_recip(s)) != __float_as_uint(exact);
        if (__float_as_uint(seed_recip(s, y)) != __float_as_uint(exact)) {
            ++bad_seed;
            const unsigned long long k = atomicAdd(&counts[3], 1ull);
            if (k < (unsigned long long)cap) list[k] = bits;
        }
    }
    if (bad_sqrt) atomicAdd(&counts[0], (unsigned long long)bad_sqrt);
    if (bad_rcp) atomicAdd(&counts[1], (unsigned long long)bad_rcp);
    if (bad_seed) atomicAdd(&counts[2], (unsigned long long)bad_seed);
}

// Sweep 2: for each listed t (blockIdx.y), every a = +-2^k * (1 + m 2^-23) with a in [s 2^-40, s]: Markstein with r'
// against IEEE a / s. counts[4] = mismatches, counts[5] = quotients tested; first_bad = the smallest failing t.
__global__ void quotient_sweep(const uint32_t* list, int n_list, unsigned long long* counts, uint32_t* first_bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23) || (int)blockIdx.y >= n_list) return;
    const float t = __uint_as_float(list[blockIdx.y]);
    float y;
    const float s = seed_sqrt(t, y);
    const float r = seed_recip(s, y);
    const int es = (int)((__float_as_uint(s) >> 23) & 0xFF);
    unsigned int bad = 0, tested = 0;
    for (int ea = es - 40; ea <= es; ++ea) {
        if (ea < 1) continue;
        const float a = __uint_as_float(((uint32_t)ea << 23) | m);
        if (a > s) continue;
        ++tested;
        bad += __float_as_uint(markstein(a, s, r)) != __float_as_uint(a / s);
        bad += __float_as_uint(markstein(-a, s, r)) != __float_as_uint(-a / s);
    }
    if (bad) {
        atomicAdd(&counts[4], (unsigned long long)bad);
        atomicMin(first_bad, list[blockIdx.y]);
    }
    atomicAdd(&counts[5], (unsigned long long)tested);
}

extern "C" int probe_seed_div(int emin, int emax, unsigned long long* out6, uint32_t* list, int cap, uint32_t* first_bad) {
    unsigned long long* d_counts;
    uint32_t *d_list, *d_first;
    if (hipMalloc(&d_counts, 6 * 8) != hipSuccess || hipMalloc(&d_list, 4 * (size_t)cap) != hipSuccess ||
        hipMalloc(&d_first, 4) != hipSuccess)
        return -1;
    (void)hipMemset(d_counts, 0, 6 * 8);
    (void)hipMemset(d_first, 0xFF, 4);
    hipLaunchKernelGGL(seed_sweep, dim3((1u << 23) / 256), dim3(256), 0, 0, emin, emax, d_counts, d_list, cap);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(out6, d_counts, 6 * 8, hipMemcpyDeviceToHost);
    const int n = out6[3] < (unsigned long long)cap ? (int)out6[3] : cap;
    if (n > 0) {
        hipLaunchKernelGGL(quotient_sweep, dim3((1u << 23) / 256, n), dim3(256), 0, 0, d_list, n, d_counts, d_first);
        if (hipDeviceSynchronize() != hipSuccess) return -3;
    }
    (void)hipMemcpy(out6, d_counts, 6 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(list, d_list, 4 * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, d_first, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_counts);
    (void)hipFree(d_list);
    (void)hipFree(d_first);
    return 0;
}
