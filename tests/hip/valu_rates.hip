// tests/hip/valu_rates.hip -- TEST-ONLY microbenchmark: issue cost of the VALU ops the shading loop
// uses (8 independent chains per lane, 256 threads/block, many blocks), and of mixes (does a
// transcendental or an fp64 op overlap packed fp32 work?). Prints SIMD-cycles per wave-instruction
// from the clock measured in-kernel (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2 __attribute__((ext_vector_type(2)));
#define N_ITER 2048

__device__ unsigned long long g_clk[2];

template <int OP>
__global__ __launch_bounds__(256) void bench(float* out, float s) {
    float a[8];
    v2 p[8];
    double d[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; p[i] = v2{a[i], a[i] + 1}; d[i] = a[i]; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
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
            if (OP == 8) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
            if (OP == 9) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
            if (OP == 10) asm volatile("v_cmp_lt_f32_e64 s[0:1], %0, %1" ::"v"(a[i]), "v"(s) : "s0", "s1");
            if (OP == 11) asm volatile("v_max_f32 %0, 0, %0" : "+v"(a[i]));
            if (OP == 12) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d[i]));
            if (OP == 13) asm volatile("v_rsq_f32 %0, %0" : "+v"(a[i]));
            if (OP == 18) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            if (OP == 19) asm volatile("v_cmp_class_f32_e64 s[0:1], %0, %1" ::"v"(a[i]), "v"(s) : "s0", "s1");
            if (OP == 20) asm volatile("v_ldexp_f32 %0, %0, 3" : "+v"(a[i]));
            if (OP == 21) asm volatile("v_med3_f32 %0, %0, %1, 1.0" : "+v"(a[i]) : "v"(s));
            if (OP == 22) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[4:5]" : "+v"(a[i]) : "v"(s));
            if (OP == 23) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            if (OP == 24) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            if (OP == 25) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            if (OP == 26) asm volatile("v_cmp_ge_u32_e64 s[0:1], %0, %1" ::"v"(a[i]), "v"(s) : "s0", "s1");
            if (OP == 27) {  // pk_fma with an s_nop in front (is the nop's slot taken by other waves?)
                asm volatile("s_nop 0\n\tv_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
            }
            if (OP == 28) asm volatile("v_pk_add_f32 %0, %0, %1 clamp" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
            // mixes: 1 transcendental per 4 packed ops, 1 fp64 mul per 4 packed ops
            if (OP == 14) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
                if ((i & 3) == 0) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
            }
            if (OP == 15) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
                if ((i & 3) == 0) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[i]));
            }
            if (OP == 16) {  // 2 unpacked fma instead of 1 packed
                asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[i]) : "v"(s));
                asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(p[i].x) : "v"(s));
            }
            if (OP == 17) {  // packed chain with its own result as the next input (dependent)
                asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p[0]));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 7 && threadIdx.x == 0) { g_clk[0] = t1 - t0; g_clk[1] = r1 - r0; }
    float r = 0;
    for (int i = 0; i < 8; ++i) r += a[i] + p[i].x + p[i].y + (float)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
static void run(const char* name, float* o, int rep, double ops_per_iter) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = 8192;
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, o, 0.999f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long clk[2];
    (void)hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
    const double ghz = clk[1] ? (double)clk[0] / (double)clk[1] * 0.1 : 2.1;
    const double waves = blocks * 256.0 / 64, ops = waves * N_ITER * ops_per_iter;
    if (rep)
        printf("%-28s %8.3f ms  clk %.2f GHz  %.2f SIMD-cycles per wave-op\n", name, ms, ghz,
               ms * 1e-3 * ghz * 1e9 * 1024 / ops);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    float* o;
    (void)hipMalloc(&o, sizeof(float) * 256 * 8192);
    for (int rep = 0; rep < 2; ++rep) {
        run<0>("v_fma_f32", o, rep, 8);
        run<6>("v_mul_f32", o, rep, 8);
        run<1>("v_pk_fma_f32", o, rep, 8);
        run<8>("v_pk_mul_f32", o, rep, 8);
        run<9>("v_pk_add_f32", o, rep, 8);
        run<16>("2x v_fma_f32 (per op)", o, rep, 16);
        run<17>("v_pk_fma_f32 dependent", o, rep, 8);
        run<2>("v_rcp_f32", o, rep, 8);
        run<13>("v_rsq_f32", o, rep, 8);
        run<4>("v_sqrt_f32", o, rep, 8);
        run<3>("v_mul_f64", o, rep, 8);
        run<12>("v_fma_f64", o, rep, 8);
        run<5>("v_cvt_f64_f32", o, rep, 8);
        run<7>("v_cndmask_b32", o, rep, 8);
        run<10>("v_cmp_lt_f32_e64 (sgpr)", o, rep, 8);
        run<11>("v_max_f32", o, rep, 8);
        run<18>("v_add_u32", o, rep, 8);
        run<19>("v_cmp_class_f32 (sgpr)", o, rep, 8);
        run<20>("v_ldexp_f32", o, rep, 8);
        run<21>("v_med3_f32", o, rep, 8);
        run<22>("v_cndmask_b32 (sgpr mask)", o, rep, 8);
        run<23>("v_and_b32", o, rep, 8);
        run<24>("v_add_f32", o, rep, 8);
        run<25>("v_max_f32 (vgpr)", o, rep, 8);
        run<26>("v_cmp_ge_u32 (sgpr)", o, rep, 8);
        run<27>("s_nop + v_pk_fma_f32", o, rep, 8);
        run<28>("v_pk_add_f32 clamp", o, rep, 8);
        run<14>("pk_fma x8 + rcp x2 (per iter)", o, rep, 1);
        run<15>("pk_fma x8 + mul_f64 x2 (iter)", o, rep, 1);
    }
    return 0;
}
