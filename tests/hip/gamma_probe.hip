// tests/hip/gamma_probe.hip -- TEST-ONLY: the accuracy of the faithful-mode gamma encode
// (pbr_device_math.h, pow_inv_gamma_faithful: v_exp_f32(kInvGamma * v_log_f32(c)) on its range,
// glibc's powf elsewhere) against the host glibc powf(c, 1.0f/2.2f), exhaustively over every float of
// each binade asked for. Built and run by tests/test_gpu_probes.py; also prints per-binade maxima.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "pbr_device_math.h"

namespace {

__global__ void k_gamma(uint32_t base, uint32_t n, float* out) {
    pbr::load_libm_tables();  // the glibc fallback reads the powf tables from LDS, as in the product kernel
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = pbr::pow_inv_gamma_faithful(__uint_as_float(base + i));
}

inline float bits_to_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

}  // namespace

// For every binade e in [e_lo, e_hi] (c in [2^e, 2^(e+1))): max relative error of the device result vs
// glibc powf, written to max_rel[e - e_lo]. Returns 0 or a HIP error code.
extern "C" int probe_gamma(int e_lo, int e_hi, double* max_rel) {
    const uint32_t n = 1u << 23;
    float* d = nullptr;
    if (hipMalloc(&d, sizeof(float) * n) != hipSuccess) return 1;
    std::vector<float> h(n);
    const float k = 1.0f / 2.2f;
    for (int e = e_lo; e <= e_hi; ++e) {
        const uint32_t base = (uint32_t)(e + 127) << 23;
        hipLaunchKernelGGL(k_gamma, dim3(n / 256), dim3(256), 0, 0, base, n, d);
        if (hipMemcpy(h.data(), d, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        const int T = 16;
        std::vector<double> part(T, 0.0);
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) {
            th.emplace_back([&, t] {
                double m = 0.0;
                for (uint32_t i = t; i < n; i += T) {
                    const float ref = powf(bits_to_float(base + i), k);
                    const double r = std::fabs((double)h[i] - (double)ref) / std::fabs((double)ref);
                    if (!(r <= m)) m = r;  // NaN propagates as a failure
                }
                part[t] = m;
            });
        }
        for (auto& x : th) x.join();
        double m = 0.0;
        for (double x : part) m = (x > m || x != x) ? x : m;
        max_rel[e - e_lo] = m;
    }
    (void)hipFree(d);
    return 0;
}
