// tests/hip/fastdiv_probe.hip -- TEST-ONLY probe of the exact fast division building blocks on gfx950.
// Built and run by tests/test_gpu_probes.py. Counts disagreements with the compiler's correctly
// rounded IEEE division (built with -fhip-fp32-correctly-rounded-divide-sqrt).
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ float recip_r1(float b) {  // v_rcp + one Newton step (fma)
    float r = __builtin_amdgcn_rcpf(b);
    float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float div_markstein(float a, float b, float y) {  // y = RN(1/b), b > 0
    float q = a * y;
    float r = __builtin_fmaf(b, q, -a);  // = -(a - b q): keeps the sign of a -0 quotient for b > 0
    return __builtin_fmaf(-r, y, q);
}
__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// (1) r1 == RN(1/b) for every significand and every exponent in [emin, emax].
__global__ void recip_exhaustive(int emin, int emax, unsigned long long* bad, unsigned int* first_bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;  // 23-bit significand
    if (m >= (1u << 23)) return;
    unsigned int nbad = 0;
    for (int e = emin; e <= emax; ++e) {
        const uint32_t bits = ((uint32_t)(e + 127) << 23) | m;
        const float b = __uint_as_float(bits);
        const float r1 = recip_r1(b);
        const float ref = 1.0f / b;
        if (__float_as_uint(r1) != __float_as_uint(ref)) {
            ++nbad;
            atomicMin(first_bad, bits);
        }
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

// (2) Markstein quotient with y = r1 on random (a, b): |a| in [2^alo, 2^ahi), b in [2^blo, 2^bhi),
// random signs for a; plus a == +-0. Counts mismatches vs a / b.
__global__ void div_random(uint64_t seed, int iters, int alo, int ahi, int blo, int bhi, unsigned long long* bad,
                           unsigned long long* bad_r1, float* example) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned int nbad = 0, nbad_r = 0;
    for (int i = 0; i < iters; ++i) {
        const uint64_t h = mix(seed ^ (t * 0x100000001B3ull + (uint64_t)i));
        const uint64_t h2 = mix(h);
        const int ea = alo + (int)((h >> 40) % (uint64_t)(ahi - alo));
        const int eb = blo + (int)((h2 >> 40) % (uint64_t)(bhi - blo));
        float a = __uint_as_float(((uint32_t)(ea + 127) << 23) | (uint32_t)(h & 0x7FFFFF));
        const float b = __uint_as_float(((uint32_t)(eb + 127) << 23) | (uint32_t)(h2 & 0x7FFFFF));
        if ((h >> 63) & 1) a = -a;
        if (((h >> 24) & 0xFFFF) == 0) a = ((h >> 62) & 1) ? -0.0f : 0.0f;
        const float y = recip_r1(b);
        const float ref = a / b;
        const float q = div_markstein(a, b, y);
        if (__float_as_uint(q) != __float_as_uint(ref)) {
            ++nbad;
            example[0] = a;
            example[1] = b;
        }
        if (__float_as_uint(y) != __float_as_uint(1.0f / b)) ++nbad_r;
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
    if (nbad_r) atomicAdd(bad_r1, (unsigned long long)nbad_r);
}

// (3) div_pi (pbr_device_math.h) == x / PI for every significand and exponent in [emin, emax].
__global__ void div_pi_exhaustive(int emin, int emax, unsigned long long* bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float pi = 3.14159265359f, zh = 0x1.45f306p-2f, zl = 0x1.11be6cp-28f;
    unsigned int nbad = 0;
    for (int e = emin; e <= emax; ++e) {
        const float x = __uint_as_float(((uint32_t)(e + 127) << 23) | m);
        if (__float_as_uint(__builtin_fmaf(x, zh, x * zl)) != __float_as_uint(x / pi)) ++nbad;
        if (__float_as_uint(__builtin_fmaf(-x, zh, -x * zl)) != __float_as_uint(-x / pi)) ++nbad;
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

extern "C" int probe_div_pi(int emin, int emax, unsigned long long* bad) {
    unsigned long long* d_bad;
    if (hipMalloc(&d_bad, 8) != hipSuccess) return -1;
    (void)hipMemset(d_bad, 0, 8);
    hipLaunchKernelGGL(div_pi_exhaustive, dim3((1u << 23) / 256), dim3(256), 0, 0, emin, emax, d_bad);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    return 0;
}

extern "C" int probe_recip(int emin, int emax, unsigned long long* bad, unsigned int* first_bad) {
    unsigned long long* d_bad;
    unsigned int* d_first;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 4) != hipSuccess) return -1;
    hipMemset(d_bad, 0, 8);
    hipMemset(d_first, 0xFF, 4);
    hipLaunchKernelGGL(recip_exhaustive, dim3((1u << 23) / 256), dim3(256), 0, 0, emin, emax, d_bad, d_first);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(first_bad, d_first, 4, hipMemcpyDeviceToHost);
    hipFree(d_bad);
    hipFree(d_first);
    return 0;
}

extern "C" int probe_div(unsigned long long seed, int blocks, int iters, int alo, int ahi, int blo, int bhi,
                         unsigned long long* bad, unsigned long long* bad_r1, float* example) {
    unsigned long long *d_bad, *d_bad_r;
    float* d_ex;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_bad_r, 8) != hipSuccess || hipMalloc(&d_ex, 8) != hipSuccess)
        return -1;
    hipMemset(d_bad, 0, 8);
    hipMemset(d_bad_r, 0, 8);
    hipMemset(d_ex, 0, 8);
    hipLaunchKernelGGL(div_random, dim3(blocks), dim3(256), 0, 0, (uint64_t)seed, iters, alo, ahi, blo, bhi, d_bad,
                       d_bad_r, d_ex);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    hipMemcpy(bad, d_bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(bad_r1, d_bad_r, 8, hipMemcpyDeviceToHost);
    hipMemcpy(example, d_ex, 8, hipMemcpyDeviceToHost);
    hipFree(d_bad);
    hipFree(d_bad_r);
    hipFree(d_ex);
    return 0;
}
