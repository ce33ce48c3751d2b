// tests/hip/valu_rates.hip -- TEST-ONLY microbenchmark: issue cost of the VALU ops the shading loop
// uses (8 independent chains per lane, 256 threads/block, many blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2 __attribute__((ext_vector_type(2)));
#define N_ITER 4096
template <int OP>
__global__ void bench(float* out, float s) {
    float a[8];
    v2 p[8];
    double d[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; p[i] = v2{a[i], a[i] + 1}; d[i] = a[i]; }
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[i]) : "v"(s));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
            if (OP == 2) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
            if (OP == 3) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[i]));
            if (OP == 4) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i]));
            if (OP == 5) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i]) : "v"(a[i]));
            if (OP == 6) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            if (OP == 7) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(s));
        }
    }
    float r = 0;
    for (int i = 0; i < 8; ++i) r += a[i] + p[i].x + p[i].y + (float)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
int main() {
    float* o;
    (void)hipMalloc(&o, sizeof(float) * 256 * 8192);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_rcp_f32", "v_mul_f64", "v_sqrt_f32", "v_cvt_f64_f32", "v_mul_f32", "v_cndmask_b32"};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep)
        for (int op = 0; op < 8; ++op) {
            (void)hipEventRecord(e0);
            const dim3 g(8192), b(256);
            switch (op) {
                case 0: hipLaunchKernelGGL(bench<0>, g, b, 0, 0, o, 0.999f); break;
                case 1: hipLaunchKernelGGL(bench<1>, g, b, 0, 0, o, 0.999f); break;
                case 2: hipLaunchKernelGGL(bench<2>, g, b, 0, 0, o, 0.999f); break;
                case 3: hipLaunchKernelGGL(bench<3>, g, b, 0, 0, o, 0.999f); break;
                case 4: hipLaunchKernelGGL(bench<4>, g, b, 0, 0, o, 0.999f); break;
                case 5: hipLaunchKernelGGL(bench<5>, g, b, 0, 0, o, 0.999f); break;
                case 6: hipLaunchKernelGGL(bench<6>, g, b, 0, 0, o, 0.999f); break;
                case 7: hipLaunchKernelGGL(bench<7>, g, b, 0, 0, o, 0.999f); break;
            }
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double waves = 8192.0 * 256 / 64, ops = waves * N_ITER * 8;
            // SIMD-cycles per wave-instruction at an assumed 2.1 GHz over 1024 SIMDs
            if (rep) printf("%-16s %8.3f ms  %.2f SIMD-cycles per wave-op (@2.1GHz)\n", names[op], ms,
                            ms * 1e-3 * 2.1e9 * 1024 / ops);
        }
    return 0;
}
