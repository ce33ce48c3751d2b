// tools/libm_x2_check.cpp -- proves the branch-free pair forms of physically_based_renderer_amd/csrc/libm_f32_x2.h
// (pbr_asinf_x2, pbr_atan2f_x2) bit-identical to the host glibc's asinf / atan2f wherever they do not report a
// special input, and that they report special inputs only where the scalar functions are needed (NaN, infinite,
// magnitudes outside [2^-40, 2^40] for atan2f; |x| > 1 for asinf). The device build evaluates the same operations
// in the same order (packed fp32 rounds each element like its scalar form; its division and square root equal
// IEEE's inside the windows the header states), so it inherits the result; tests/hip/libm_probe.hip checks the
// device build directly on the GPU.
//   asinf:          every float in [-1, 1] (pairs of neighbours), plus every float above 1 (special)
//   atan2f(y, 1):   every finite y (the atanf core and the x == 1 case)
//   atan2f(y, x):   2e9 random pairs -- unit directions as WorldToSkyUV sees them, near-axis and near-zero
//                   components, random bit patterns, signed zeros
//
//   /opt/rocm/llvm/bin/clang++ -std=c++17 -O2 -ffp-contract=off -fno-builtin -I physically_based_renderer_amd/csrc \
//       tools/libm_x2_check.cpp -o build/libm_x2_check -lm -lpthread && build/libm_x2_check
// `--quick` sweeps every 61st bit pattern and 2e7 pairs (tests/test_host.py runs that).
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define LIBM_F32_HOST 1
#include "libm_f32_x2.h"

static const pbr_atan_seg kTab[5] = PBR_ATAN_SEG_TABLE_INIT;

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline int same(float a, float b) { return fbits(a) == fbits(b) || (a != a && b != b); }

static uint64_t g_stride = 1;
static uint64_t g_pairs = 2000000000ull;

static inline uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Pair i of the random set: directions (components in [-1, 1], some scaled towards 0 or exactly 0), signed zeros,
// and raw bit patterns.
static inline void pair(uint64_t i, float& y, float& x) {
    const uint64_t h = mix(0x5eed ^ (i * 0x100000001B3ull));
    const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
    switch (i & 7) {
        case 0: y = bitsf(lo); x = bitsf(hi); break;
        case 1: y = bitsf(lo); x = (hi & 1) ? 1.0f : -1.0f; break;
        case 2: y = (lo & 1) ? 0.0f : -0.0f; x = (float)(hi >> 8) * 0x1p-23f - 1.0f; break;
        case 3: y = (float)(lo >> 8) * 0x1p-23f - 1.0f; x = (hi & 1) ? 0.0f : -0.0f; break;
        default: {
            const float a = (float)(lo >> 8) * 0x1p-23f - 1.0f, b = (float)(hi >> 8) * 0x1p-23f - 1.0f;
            const int sh = (int)((h >> 20) & 63);
            y = (i & 8) ? ldexpf(a, -sh) : a;
            x = (i & 16) ? ldexpf(b, -sh) : b;
        }
    }
}

struct Job {
    uint64_t lo, hi, bad, bad_special, specials;
    uint32_t first;
    int what;
};

static void* run(void* p) {
    Job* j = (Job*)p;
    for (uint64_t u = j->lo; u < j->hi; u += 2 * g_stride) {
        float in0, in1, y0, y1;
        pbr_lv2 got;
        float want[2];
        int special[2];
        if (j->what == 0) {  // asinf on neighbouring bit patterns
            in0 = bitsf((uint32_t)u);
            in1 = bitsf((uint32_t)(u + 1));
            got = pbr_asinf_x2((pbr_lv2){in0, in1}, special);
            want[0] = asinf(in0);
            want[1] = asinf(in1);
            const int need[2] = {fabsf(in0) > 1.0f || in0 != in0, fabsf(in1) > 1.0f || in1 != in1};
            for (int e = 0; e < 2; ++e) {
                if (special[e] != need[e]) ++j->bad_special;
                j->specials += special[e];
            }
        } else if (j->what == 1) {  // atan2f(y, 1)
            in0 = bitsf((uint32_t)u);
            in1 = bitsf((uint32_t)(u + 1));
            got = pbr_atan2f_x2((pbr_lv2){in0, in1}, (pbr_lv2)(1.0f), special, kTab);
            want[0] = atan2f(in0, 1.0f);
            want[1] = atan2f(in1, 1.0f);
            for (int e = 0; e < 2; ++e) {
                const float v = e ? in1 : in0;
                const float a = fabsf(v);
                const int need = !(a == 0.0f || (a >= 0x1p-40f && a <= 0x1p40f));
                if (special[e] != need) ++j->bad_special;
                j->specials += special[e];
            }
        } else {  // random atan2f pairs
            pair(u, y0, in0);
            pair(u + 1, y1, in1);
            got = pbr_atan2f_x2((pbr_lv2){y0, y1}, (pbr_lv2){in0, in1}, special, kTab);
            want[0] = atan2f(y0, in0);
            want[1] = atan2f(y1, in1);
            for (int e = 0; e < 2; ++e) {
                const float ya = fabsf(e ? y1 : y0), xa = fabsf(e ? in1 : in0);
                const int need = !((ya == 0.0f || (ya >= 0x1p-40f && ya <= 0x1p40f)) &&
                                   (xa == 0.0f || (xa >= 0x1p-40f && xa <= 0x1p40f)));
                if (special[e] != need) ++j->bad_special;
                j->specials += special[e];
            }
        }
        for (int e = 0; e < 2; ++e) {
            if (special[e]) continue;  // the caller takes the scalar function there
            if (!same(e ? got.y : got.x, want[e])) {
                if (!j->bad) j->first = j->what == 2 ? (uint32_t)(u + e) : fbits(e ? in1 : in0);
                ++j->bad;
            }
        }
    }
    return nullptr;
}

static int sweep(int what, uint64_t lo, uint64_t hi, const char* name) {
    const int T = 8;
    pthread_t th[T];
    Job jobs[T];
    uint64_t n = hi - lo;
    for (int t = 0; t < T; ++t) {
        uint64_t a = lo + n * t / T, b = lo + n * (t + 1) / T;
        a -= (a - lo) % (2 * g_stride);  // keep the pairs aligned
        jobs[t] = Job{a, b, 0, 0, 0, 0xffffffffu, what};
        pthread_create(&th[t], nullptr, run, &jobs[t]);
    }
    uint64_t bad = 0, bad_special = 0, specials = 0;
    uint32_t first = 0xffffffffu;
    for (int t = 0; t < T; ++t) {
        pthread_join(th[t], nullptr);
        bad += jobs[t].bad;
        bad_special += jobs[t].bad_special;
        specials += jobs[t].specials;
        if (jobs[t].bad && first == 0xffffffffu) first = jobs[t].first;
    }
    printf("%-26s %12llu mismatches  %llu special-flag errors  (%llu special)  first 0x%08x\n", name,
           (unsigned long long)bad, (unsigned long long)bad_special, (unsigned long long)specials, first);
    return bad != 0 || bad_special != 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && !strcmp(argv[1], "--quick")) {
        g_stride = 61;
        g_pairs = 20000000ull;
    }
    int fail = 0;
    // asinf: [-1, 1] and the specials above 1 (both signs); every bit pattern from 0 to 0x80000000 + 1.0f + a
    // stretch beyond, in neighbouring pairs.
    fail |= sweep(0, 0x00000000ull, 0x3f800000ull + 0x1000000ull, "asinf x2 (+, to 1 and past)");
    fail |= sweep(0, 0x80000000ull, 0xbf800000ull + 0x1000000ull, "asinf x2 (-, to -1 and past)");
    // atan2f(y, 1): every finite y of either sign
    fail |= sweep(1, 0x00000000ull, 0x7f800000ull, "atan2f x2 (y, 1), y >= +0");
    fail |= sweep(1, 0x80000000ull, 0xff800000ull, "atan2f x2 (y, 1), y <= -0");
    fail |= sweep(2, 0, g_pairs, "atan2f x2 random pairs");
    printf(fail ? "FAIL\n" : "OK\n");
    return fail;
}
