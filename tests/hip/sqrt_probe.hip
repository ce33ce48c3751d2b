// tests/hip/sqrt_probe.hip -- TEST-ONLY probe: which cheap sqrt sequences on gfx950 equal IEEE sqrtf
// (built with -fhip-fp32-correctly-rounded-divide-sqrt) for every float with exponent in [emin, emax].
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ float cand(int which, float x) {
    switch (which) {
        case 0: return __builtin_amdgcn_sqrtf(x);  // bare v_sqrt_f32
        case 1: {                                  // rsq + one Newton/Goldschmidt step
            const float y = __builtin_amdgcn_rsqf(x);
            const float s0 = x * y;
            const float r = __builtin_fmaf(-s0, s0, x);
            return __builtin_fmaf(r, 0.5f * y, s0);
        }
        case 2: {                                  // v_sqrt + one correction step with rsq
            const float s0 = __builtin_amdgcn_sqrtf(x);
            const float y = __builtin_amdgcn_rsqf(x);
            const float r = __builtin_fmaf(-s0, s0, x);
            return __builtin_fmaf(r, 0.5f * y, s0);
        }
        default: {                                 // v_sqrt + one correction step with rcp(s0)
            const float s0 = __builtin_amdgcn_sqrtf(x);
            const float r = __builtin_fmaf(-s0, s0, x);
            return __builtin_fmaf(r, 0.5f * __builtin_amdgcn_rcpf(s0), s0);
        }
    }
}

__global__ void sqrt_sweep(int which, int emin, int emax, unsigned long long* bad, unsigned int* first_bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;  // 23-bit significand
    if (m >= (1u << 23)) return;
    unsigned int nbad = 0;
    for (int e = emin; e <= emax; ++e) {
        const uint32_t bits = ((uint32_t)(e + 127) << 23) | m;
        const float x = __uint_as_float(bits);
        if (__float_as_uint(cand(which, x)) != __float_as_uint(sqrtf(x))) {
            ++nbad;
            atomicMin(first_bad, bits);
        }
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

// RN(1 / RN(sqrt(t))) from the rsq seed the sqrt already computed: one Newton step on the rounded s.
__global__ void recip_sqrt_sweep(int which, int emin, int emax, unsigned long long* bad, unsigned int* first_bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    unsigned int nbad = 0;
    for (int e = emin; e <= emax; ++e) {
        const uint32_t bits = ((uint32_t)(e + 127) << 23) | m;
        const float t = __uint_as_float(bits);
        const float y = __builtin_amdgcn_rsqf(t);
        const float s0 = t * y;
        const float s = __builtin_fmaf(__builtin_fmaf(-s0, s0, t), 0.5f * y, s0);
        float r;
        if (which == 0) {  // Newton on 1/s from y
            r = __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y);
        } else if (which == 2) {  // two Newton steps on 1/s from y (no v_rcp)
            const float r1 = __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y);
            r = __builtin_fmaf(__builtin_fmaf(-s, r1, 1.0f), r1, r1);
        } else {           // control: v_rcp(s) + Newton (the current path)
            const float r0 = __builtin_amdgcn_rcpf(s);
            r = __builtin_fmaf(__builtin_fmaf(-s, r0, 1.0f), r0, r0);
        }
        if (__float_as_uint(r) != __float_as_uint(1.0f / s)) {
            ++nbad;
            atomicMin(first_bad, bits);
        }
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

extern "C" int probe_recip_sqrt(int which, int emin, int emax, unsigned long long* bad, unsigned int* first_bad) {
    unsigned long long* d_bad;
    unsigned int* d_first;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 4) != hipSuccess) return -1;
    (void)hipMemset(d_bad, 0, 8);
    (void)hipMemset(d_first, 0xFF, 4);
    hipLaunchKernelGGL(recip_sqrt_sweep, dim3((1u << 23) / 256), dim3(256), 0, 0, which, emin, emax, d_bad, d_first);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, d_first, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return 0;
}

extern "C" int probe_sqrt(int which, int emin, int emax, unsigned long long* bad, unsigned int* first_bad) {
    unsigned long long* d_bad;
    unsigned int* d_first;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 4) != hipSuccess) return -1;
    (void)hipMemset(d_bad, 0, 8);
    (void)hipMemset(d_first, 0xFF, 4);
    hipLaunchKernelGGL(sqrt_sweep, dim3((1u << 23) / 256), dim3(256), 0, 0, which, emin, emax, d_bad, d_first);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, d_first, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return 0;
}
