// tests/hip/rsq_recip_probe.hip -- TEST-ONLY probe: RN(1 / s) for s = RN(sqrt(t)) (the kernel's sqrt_nr) from the
// v_rsq seed y the square root already computed, in three fused operations instead of a v_rcp (8 SIMD cycles per
// element) and a Newton step. Every t with exponent in [emin, emax] is tried; a candidate must equal the IEEE
// quotient 1.0f / s bit for bit. Variants:
//   0  control: v_rcp(s), one Newton step (the kernels' recip_nr)
//   1  one Newton step from y:             e = 1 - s y;  r = y + e y
//   2  two Newton steps from y (4 ops; round 3 found it one ulp low at s with an all-ones significand)
//   3  Newton with the second-order term:  e = 1 - s y;  c = e + e^2;  r = y + c y
//   4  Newton with the refined product:    e = 1 - s y;  r1 = y + e y;  r = y + e r1
//   5  one Newton step from the seed nudged one ulp up
//   6  one Newton step with the correction scaled by 1 + 2^-23
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ float sqrt_seed(float t, float& y) {
    y = __builtin_amdgcn_rsqf(t);
    const float s0 = t * y;
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, t), 0.5f * y, s0);
}

__device__ __forceinline__ float cand(int which, float s, float y) {
    switch (which) {
        case 0: {
            const float r0 = __builtin_amdgcn_rcpf(s);
            return __builtin_fmaf(__builtin_fmaf(-s, r0, 1.0f), r0, r0);
        }
        case 1:
            return __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y);
        case 2: {
            const float r1 = __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y);
            return __builtin_fmaf(__builtin_fmaf(-s, r1, 1.0f), r1, r1);
        }
        case 3: {
            const float e = __builtin_fmaf(-s, y, 1.0f);
            return __builtin_fmaf(__builtin_fmaf(e, e, e), y, y);
        }
        case 4: {
            const float e = __builtin_fmaf(-s, y, 1.0f);
            const float r1 = __builtin_fmaf(e, y, y);
            return __builtin_fmaf(e, r1, y);
        }
        case 5: {  // seed nudged one ulp up
            const float yb = y * 0x1.000002p0f;
            return __builtin_fmaf(__builtin_fmaf(-s, yb, 1.0f), yb, yb);
        }
        default: {  // correction scaled by 1 + 2^-23
            const float e = __builtin_fmaf(-s, y, 1.0f);
            return __builtin_fmaf(__builtin_fmaf(e, 0x1p-23f, e), y, y);
        }
    }
}

__global__ void rsq_recip_sweep(int which, int emin, int emax, unsigned long long* bad, uint32_t* log, int nlog) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;  // 23-bit significand of t
    if (m >= (1u << 23)) return;
    unsigned int nbad = 0;
    for (int e = emin; e <= emax; ++e) {
        const float t = __uint_as_float(((uint32_t)(e + 127) << 23) | m);
        float y;
        const float s = sqrt_seed(t, y);
        const float r = cand(which, s, y);
        const float want = 1.0f / s;  // IEEE (built with -fhip-fp32-correctly-rounded-divide-sqrt)
        if (__float_as_uint(r) != __float_as_uint(want)) {
            ++nbad;
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < (unsigned long long)nlog) {
                log[4 * k] = __float_as_uint(t);
                log[4 * k + 1] = __float_as_uint(s);
                log[4 * k + 2] = __float_as_uint(r);
                log[4 * k + 3] = __float_as_uint(want);
            }
        }
    }
    (void)nbad;
}

extern "C" int probe_rsq_recip(int which, int emin, int emax, unsigned long long* bad, uint32_t* log, int nlog) {
    unsigned long long* d_bad;
    uint32_t* d_log;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_log, 16 * (size_t)(nlog > 0 ? nlog : 1)) != hipSuccess)
        return -1;
    (void)hipMemset(d_bad, 0, 8);
    hipLaunchKernelGGL(rsq_recip_sweep, dim3((1u << 23) / 256), dim3(256), 0, 0, which, emin, emax, d_bad, d_log, nlog);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    if (nlog > 0) (void)hipMemcpy(log, d_log, 16 * (size_t)nlog, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    (void)hipFree(d_log);
    return 0;
}
