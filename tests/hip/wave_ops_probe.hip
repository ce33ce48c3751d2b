// tests/hip/wave_ops_probe.hip -- TEST-ONLY probe: the DPP wave reductions and scan of pbr_device_math_x2.h
// (wave_min_dpp, wave_max_dpp, wave_sum_dpp, wave_scan_add_dpp) on many waves of host-chosen values, for
// tests/test_gpu_probes.py to compare with a serial evaluation (NaN inputs count as the neutral value).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "pbr_device_math_x2.h"

__global__ void wave_ops_kernel(const float* __restrict__ f, const int* __restrict__ iv, float* out_min,
                                float* out_max, int* out_sum, int* out_scan) {
    const int w = blockIdx.x, l = threadIdx.x;
    const float v = f[64 * w + l];
    const int k = iv[64 * w + l];
    const float mn = pbr::wave_min_dpp(v), mx = pbr::wave_max_dpp(v);
    const int sm = pbr::wave_sum_dpp(k);
    out_scan[64 * w + l] = pbr::wave_scan_add_dpp(k);
    if (l == 0) {
        out_min[w] = mn;
        out_max[w] = mx;
        out_sum[w] = sm;
    }
}

extern "C" int probe_wave_ops(const float* f, const int* iv, int n_waves, float* out_min, float* out_max, int* out_sum,
                              int* out_scan) {
    float *df, *dmin, *dmax;
    int *di, *dsum, *dscan;
    const size_t n = (size_t)64 * n_waves;
    if (hipMalloc(&df, n * 4) != hipSuccess || hipMalloc(&di, n * 4) != hipSuccess ||
        hipMalloc(&dmin, 4 * (size_t)n_waves) != hipSuccess || hipMalloc(&dmax, 4 * (size_t)n_waves) != hipSuccess ||
        hipMalloc(&dsum, 4 * (size_t)n_waves) != hipSuccess || hipMalloc(&dscan, n * 4) != hipSuccess)
        return -1;
    (void)hipMemcpy(df, f, n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(di, iv, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(wave_ops_kernel, dim3(n_waves), dim3(64), 0, 0, df, di, dmin, dmax, dsum, dscan);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    (void)hipMemcpy(out_min, dmin, 4 * (size_t)n_waves, hipMemcpyDeviceToHost);
    (void)hipMemcpy(out_max, dmax, 4 * (size_t)n_waves, hipMemcpyDeviceToHost);
    (void)hipMemcpy(out_sum, dsum, 4 * (size_t)n_waves, hipMemcpyDeviceToHost);
    (void)hipMemcpy(out_scan, dscan, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(df);
    (void)hipFree(di);
    (void)hipFree(dmin);
    (void)hipFree(dmax);
    (void)hipFree(dsum);
    (void)hipFree(dscan);
    return 0;
}
