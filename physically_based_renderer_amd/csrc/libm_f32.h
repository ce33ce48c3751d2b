/* libm_f32.h -- fp32 atan2f, asinf and powf with the exact operation sequences of the host C
 * library the oracle runs on, for device and host:
 *   atan2f/asinf: glibc 2.35 sysdeps/ieee754/flt-32 (e_atan2f.c + s_atanf.c, the fdlibm float
 *                 conversion; e_asinf.c, the Cephes-polynomial version);
 *   powf:         glibc 2.35's x86-64 FMA variant (sysdeps/ieee754/flt-32/e_powf.c built with
 *                 -mfma -mavx2, selected by ifunc on every FMA-capable x86-64 host): log2 through a
 *                 16-entry (1/c, log2 c) table and a degree-4 polynomial, exp2 through a 32-entry
 *                 2^(i/32) table and a degree-2 polynomial, all in fp64 with the FMAs that build has.
 *
 * Why: the reference's WorldToSkyUV (LightingUtil.hlsl:216-225) maps a direction to the sky texture
 * through atan2 and asin; near the poles (|N.y| -> 1) asin is so steep that a one-ulp difference in
 * either function moves the sampled texel by a visible fraction and the shaded colour by up to
 * 1.6e-4 relative -- well past the 1e-5 parity bar. The device library's (ocml) functions are
 * faithfully rounded but not the same function as glibc's, so the kernel evaluates this port
 * instead: IEEE add/mul/div/sqrt in the same order, never contracted, gives the same bits on both
 * sides. tools/libm_port_check.c proves the host restatement bit-identical to glibc (exhaustively
 * for asinf on [-1, 1] and atanf on every finite float, plus 2e9 random atan2f pairs).
 *
 * Host builds need -ffp-contract=off; device bodies turn contraction off themselves.
 */
#ifndef PBR_LIBM_F32_H
#define PBR_LIBM_F32_H

#ifdef LIBM_F32_HOST
#include <stdint.h>
#include <string.h>
#include <math.h>
#define PBR_LIBM_FN static inline
static inline uint32_t pbr_lm_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float pbr_lm_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
#define PBR_LM_SQRTF(x) sqrtf(x)
#define PBR_LM_FABSF(x) fabsf(x)
#define PBR_LM_NO_CONTRACT
#else
#define PBR_LIBM_FN __device__ __forceinline__
__device__ __forceinline__ uint32_t pbr_lm_bits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float pbr_lm_float(uint32_t u) { return __uint_as_float(u); }
#define PBR_LM_SQRTF(x) sqrtf(x) /* correctly rounded under -fhip-fp32-correctly-rounded-divide-sqrt; __fsqrt_rn is not */
#define PBR_LM_FABSF(x) __builtin_fabsf(x)
#define PBR_LM_NO_CONTRACT _Pragma("clang fp contract(off)")
#endif

/* |y/x| exponent gap beyond which atan2f returns +-pi/2 (or 0 for x < 0) without dividing. */
#ifndef PBR_ATAN2F_KMAX
#define PBR_ATAN2F_KMAX 26
#endif

/* ---- powf ---------------------------------------------------------------------------------- */

typedef struct { double invc, logc; } pbr_powf_log2_entry;

/* The published tables of the algorithm (identical to the host library's .rodata). */
#define PBR_POWF_LOG2_TABLE_INIT { \
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2}, \
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2}, \
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3}, \
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4}, \
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0}, \
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3}, \
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2}, \
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}}
#define PBR_EXP2F_TABLE_INIT { \
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull, \
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull, \
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull, \
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull, \
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull, \
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull, \
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull, \
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

#ifdef LIBM_F32_HOST
static const pbr_powf_log2_entry pbr_powf_log2_tab[16] = PBR_POWF_LOG2_TABLE_INIT;
static const uint64_t pbr_exp2f_tab[32] = PBR_EXP2F_TABLE_INIT;
#define PBR_LM_FMA(a, b, c) fma(a, b, c)
static inline uint64_t pbr_lm_bits64(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double pbr_lm_double(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
#else
static __constant__ pbr_powf_log2_entry pbr_powf_log2_tab[16] = PBR_POWF_LOG2_TABLE_INIT;
static __constant__ uint64_t pbr_exp2f_tab[32] = PBR_EXP2F_TABLE_INIT;
#define PBR_LM_FMA(a, b, c) __builtin_fma(a, b, c)
__device__ __forceinline__ uint64_t pbr_lm_bits64(double d) { return __double_as_longlong(d); }
__device__ __forceinline__ double pbr_lm_double(uint64_t u) { return __longlong_as_double(u); }
#endif

#define PBR_POWF_SIGN_BIAS 0x10000u /* 1 << (5 + 11) */

/* log2(x) for the normalised positive bit pattern ix (log2_inline). */
PBR_LIBM_FN double pbr_powf_log2(uint32_t ix, const pbr_powf_log2_entry* tab) {
    PBR_LM_NO_CONTRACT
    const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                 A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp+0;
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double z = (double)pbr_lm_float(iz);
    const double r = PBR_LM_FMA(z, tab[i].invc, -1.0);
    const double y0 = (double)k + tab[i].logc;
    const double y = PBR_LM_FMA(r, A0, A1);
    const double p = PBR_LM_FMA(r, A2, A3);
    const double r2 = r * r;
    double q = PBR_LM_FMA(r, A4, y0);
    const double r4 = r2 * r2;
    q = PBR_LM_FMA(r2, p, q);
    return PBR_LM_FMA(y, r4, q);
}

/* 2^xd rounded to float, sign from sign_bias (exp2_inline). */
PBR_LIBM_FN float pbr_powf_exp2(double xd, uint32_t sign_bias, const uint64_t* tab) {
    PBR_LM_NO_CONTRACT
    const double SHIFT = 0x1.8p+47, C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3,
                 C2 = 0x1.62e42ff0c52d6p-1;
    double kd = xd + SHIFT;
    const uint64_t ki = pbr_lm_bits64(kd);
    kd -= SHIFT;
    const double r = xd - kd;
    const uint64_t t = tab[ki & 31u] + ((ki + sign_bias) << 47);
    const double s = pbr_lm_double(t);
    const double z = PBR_LM_FMA(r, C0, C1);
    const double r2 = r * r;
    double y = PBR_LM_FMA(r, C2, 1.0);
    y = PBR_LM_FMA(z, r2, y);
    y = y * s;
    return (float)y;
}

/* 0: not an integer, 1: odd integer, 2: even integer (checkint). */
PBR_LIBM_FN int pbr_powf_checkint(uint32_t iy) {
    const int e = (int)((iy >> 23) & 0xffu);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1u)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}

PBR_LIBM_FN int pbr_powf_zeroinfnan(uint32_t i) { return 2u * i - 1u >= 2u * 0x7f800000u - 1u; }
PBR_LIBM_FN int pbr_powf_issignaling(uint32_t i) { return ((i ^ 0x00400000u) & 0x7fffffffu) > 0x7fc00000u; }
/* __math_xflowf: (sign ? -c : c) * c, rounded to float. */
PBR_LIBM_FN float pbr_powf_xflow(uint32_t sign, float c) { return (sign ? -c : c) * c; }

/* powf(x, y) with explicit tables (the device passes an LDS copy). */
PBR_LIBM_FN float pbr_powf_tab(float x, float y, const pbr_powf_log2_entry* ltab, const uint64_t* etab) {
    PBR_LM_NO_CONTRACT
    uint32_t sign_bias = 0;
    uint32_t ix = pbr_lm_bits(x);
    const uint32_t iy = pbr_lm_bits(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || pbr_powf_zeroinfnan(iy)) {
        if (pbr_powf_zeroinfnan(iy)) {
            if (2u * iy == 0) return pbr_powf_issignaling(ix) ? x + y : 1.0f;
            if (ix == 0x3f800000u) return pbr_powf_issignaling(iy) ? x + y : 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (pbr_powf_zeroinfnan(ix)) {
            float x2 = x * x;
            uint32_t neg = 0;
            if ((ix & 0x80000000u) && pbr_powf_checkint(iy) == 1) {
                x2 = -x2;
                neg = 1;
            }
            if (2u * ix == 0 && (iy & 0x80000000u)) return (neg ? -1.0f : 1.0f) / 0.0f;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) { /* finite x < 0 */
            const int yint = pbr_powf_checkint(iy);
            if (yint == 0) return (x - x) / (x - x);
            if (yint == 1) sign_bias = PBR_POWF_SIGN_BIAS;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) { /* subnormal x: normalise */
            ix = pbr_lm_bits(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = pbr_powf_log2(ix, ltab);
    const double ylogx = (double)y * logx;
    if (((pbr_lm_bits64(ylogx) >> 47) & 0xffffu) >= (0x405F800000000000ull >> 47)) { /* |ylogx| >= 126 */
        if (ylogx > 0x1.fffffffd1d571p+6) return pbr_powf_xflow(sign_bias, 0x1p97f);
        if (ylogx <= -150.0) return pbr_powf_xflow(sign_bias, 0x1p-95f);
        if (ylogx < -149.0) return pbr_powf_xflow(sign_bias, 0x1.4p-75f);
    }
    return pbr_powf_exp2(ylogx, sign_bias, etab);
}

PBR_LIBM_FN float pbr_powf(float x, float y) { return pbr_powf_tab(x, y, pbr_powf_log2_tab, pbr_exp2f_tab); }

/* powf(x, 5.0f) for x in {+0} U [2^-24, 1] -- Schlick's (1 - cos)^5 with cos = saturate(.) -- where
 * none of powf's special cases but x == 0 can occur and |5 log2 x| <= 120 < 126. */
PBR_LIBM_FN float pbr_pow5_unit(float x, const pbr_powf_log2_entry* ltab, const uint64_t* etab) {
    PBR_LM_NO_CONTRACT
    if (x == 0.0f) return 0.0f;
    return pbr_powf_exp2(5.0 * pbr_powf_log2(pbr_lm_bits(x), ltab), 0, etab);
}

/* ---- atan2f / asinf ------------------------------------------------------------------------- */

/* atanf on the reduced ranges (s_atanf.c): 4 breakpoints, odd/even split polynomial. */
PBR_LIBM_FN float pbr_atanf(float x) {
    PBR_LM_NO_CONTRACT
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
                atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
                atanlo3 = 7.5497894159e-08f;
    const float a0 = 3.3333334327e-01f, a1 = -2.0000000298e-01f, a2 = 1.4285714924e-01f,
                a3 = -1.1111110449e-01f, a4 = 9.0908870101e-02f, a5 = -7.6918758452e-02f,
                a6 = 6.6610731184e-02f, a7 = -5.8335702866e-02f, a8 = 4.9768779427e-02f,
                a9 = -3.6531571299e-02f, a10 = 1.6285819933e-02f;
    const uint32_t hx = pbr_lm_bits(x), ix = hx & 0x7fffffffu;
    const int neg = (hx >> 31) != 0;
    float hi, lo;
    int id;
    if (ix >= 0x4c000000u) { /* |x| >= 2^25 */
        if (ix > 0x7f800000u) return x + x;
        return neg ? -atanhi3 - atanlo3 : atanhi3 + atanlo3;
    }
    if (ix < 0x3ee00000u) { /* |x| < 0.4375 */
        if (ix < 0x31000000u) return x; /* |x| < 2^-29 */
        id = -1;
        hi = lo = 0.0f;
    } else {
        x = PBR_LM_FABSF(x);
        if (ix < 0x3f980000u) {        /* |x| < 1.1875 */
            if (ix < 0x3f300000u) {    /* 7/16 <= |x| < 11/16 */
                id = 0; hi = atanhi0; lo = atanlo0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {                   /* 11/16 <= |x| < 19/16 */
                id = 1; hi = atanhi1; lo = atanlo1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000u) { /* |x| < 2.4375 */
            id = 2; hi = atanhi2; lo = atanlo2;
            x = (x - 1.5f) / (1.0f + 1.5f * x);
        } else {                       /* 2.4375 <= |x| < 2^25 */
            id = 3; hi = atanhi3; lo = atanlo3;
            x = -1.0f / x;
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
    const float s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = hi - ((x * (s1 + s2) - lo) - x);
    return neg ? -r : r;
}

/* atan2f (e_atan2f.c): special cases, quadrant from the signs, atanf of |y/x|. */
PBR_LIBM_FN float pbr_atan2f(float y, float x) {
    PBR_LM_NO_CONTRACT
    const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f, tiny = 1.0e-30f;
    const uint32_t hx = pbr_lm_bits(x), ix = hx & 0x7fffffffu;
    const uint32_t hy = pbr_lm_bits(y), iy = hy & 0x7fffffffu;
    if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;
    if (hx == 0x3f800000u) return pbr_atanf(y);
    const int m = (int)((hy >> 31) & 1u) | (int)((hx >> 30) & 2u);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy >> 31) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000u) {
        if (iy == 0x7f800000u) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000u) return (hy >> 31) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = ((int)iy - (int)ix) >> 23;
    float z;
    if (k > PBR_ATAN2F_KMAX) z = pi_o_2 + 0.5f * pi_lo;
    else if ((hx >> 31) && k < -PBR_ATAN2F_KMAX) z = 0.0f;
    else z = pbr_atanf(PBR_LM_FABSF(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

/* asinf (e_asinf.c): x + x^3 P(x^2) below 0.5, half-angle reduction with a split sqrt above. */
PBR_LIBM_FN float pbr_asinf(float x) {
    PBR_LM_NO_CONTRACT
    const float pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
                pio4_hi = 0.785398185253143310546875f;
    const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                p4 = 4.216630880e-2f;
    const uint32_t hx = pbr_lm_bits(x), ix = hx & 0x7fffffffu;
    if (ix == 0x3f800000u) return x * pio2_hi + x * pio2_lo;
    if (ix > 0x3f800000u) return (x - x) / (x - x);
    if (ix < 0x3f000000u) { /* |x| < 0.5 */
        if (ix < 0x32000000u) return x;
        const float t = x * x;
        const float w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
        return x + x * w;
    }
    float w = 1.0f - PBR_LM_FABSF(x);
    float t = w * 0.5f;
    float p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    const float s = PBR_LM_SQRTF(t);
    if (ix >= 0x3f79999au) { /* |x| > 0.975 */
        t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
    } else {
        w = pbr_lm_float(pbr_lm_bits(s) & 0xfffff000u);
        const float c = (t - w * w) / (s + w);
        const float r = p;
        p = 2.0f * s * r - (pio2_lo - 2.0f * c);
        const float q = pio4_hi - 2.0f * w;
        t = pio4_hi - (p - q);
    }
    return (hx >> 31) ? -t : t;
}

#endif /* PBR_LIBM_F32_H */
