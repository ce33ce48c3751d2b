/* libm_f32_x2.h -- WorldToSkyUV's atan2f and asinf (libm_f32.h: glibc 2.35's flt-32 e_atan2f.c + s_atanf.c and
 * e_asinf.c) for a PAIR of arguments at once, without branches, bit for bit the same as the scalar restatement.
 *
 * Why: the scalar functions branch on the argument's range (atanf: five reduction intervals, each with its own
 * IEEE division; asinf: two regimes and a sub-case). With the uncorrelated normals of a G-buffer every branch
 * runs in every wave, one pixel at a time: the diffuse-IBL block was 1,054 VALU instructions per wave of the
 * headline kernel (14% of all; tools/variant_pmc.sh). Here every interval's operands are selected
 * per element first and ONE chain of operations runs for both pixels in packed fp32 (v_pk_mul/add/fma_f32): the
 * same IEEE operations in the same order as the branch the element would have taken, so the same bits:
 *   atanf reduction x' = RN(RN(A x) - C) / RN(RN(C x) + A), rounded as the branch rounds it (table rows below):
 *     |x| < 7/16: A = 1, C = 0 -> x / 1 = x;  < 11/16: (2x - 1) / (x + 2);  < 19/16: (x - 1) / (x + 1);
 *     < 39/16: (x - 1.5) / (1.5x + 1);  else: (0x - 1) / (x + 0) = -1 / x   (RN(A x) is exact or the branch's own
 *     product, and adding 0 or multiplying by 1 changes nothing);
 *   result hi - ((x' S - lo) - x'), which for the first interval (hi = lo = 0) is RN(x' - RN(x' S)), the branch's
 *   x - x S, by the symmetry of round-to-nearest.
 * Special inputs the selects do not cover -- NaN or infinite components, nonzero magnitudes outside
 * [2^-40, 2^40] (atan2f), |x| > 1 (asinf) -- are reported in `special`; the caller then takes the scalar functions
 * for the wave (tests/hip/libm_probe.hip and tools/libm_x2_check.cpp compare both against glibc).
 *
 * Divisions and the square root: on the device the exact fast sequences (Markstein division on a v_rcp + Newton
 * reciprocal, rsq + Newton sqrt), whose operands stay inside their proven windows here (comments below); the host
 * build (LIBM_F32_HOST, the CPU check) uses IEEE / and sqrtf, which those sequences equal in the window.
 */
#ifndef PBR_LIBM_F32_X2_H
#define PBR_LIBM_F32_X2_H

#include "libm_f32.h"

typedef float pbr_lv2 __attribute__((ext_vector_type(2)));

#ifdef LIBM_F32_HOST
#define PBR_LX2_FN static inline
PBR_LX2_FN pbr_lv2 pbr_lx2_div(pbr_lv2 a, pbr_lv2 b) { return a / b; }
PBR_LX2_FN pbr_lv2 pbr_lx2_sqrt(pbr_lv2 a) { return (pbr_lv2){sqrtf(a.x), sqrtf(a.y)}; }
#else
#define PBR_LX2_FN __device__ __forceinline__
/* a / b, correctly rounded, for b in [2^-60, 2^60], a == 0 or |a| in [2^-96, 2^60], |a / b| in [2^-120, 2^120]
 * (pbr_device_math.h: recip_nr is RN(1/b) there, and the Markstein step gives RN(a/b)). */
PBR_LX2_FN pbr_lv2 pbr_lx2_div(pbr_lv2 a, pbr_lv2 b) {
    const pbr_lv2 r0 = (pbr_lv2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    const pbr_lv2 e = __builtin_elementwise_fma(-b, r0, (pbr_lv2)(1.0f));
    const pbr_lv2 r = __builtin_elementwise_fma(e, r0, r0);
    const pbr_lv2 q = a * r;
    const pbr_lv2 t = __builtin_elementwise_fma(b, q, -a);
    return __builtin_elementwise_fma(-t, r, q);
}
/* sqrtf for exponents in [-64, 64] (pbr_device_math.h sqrt_nr, probed on gfx950). */
PBR_LX2_FN pbr_lv2 pbr_lx2_sqrt(pbr_lv2 x) {
    const pbr_lv2 y = (pbr_lv2){__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)};
    const pbr_lv2 s0 = x * y;
    const pbr_lv2 r = __builtin_elementwise_fma(-s0, s0, x);
    return __builtin_elementwise_fma(r, 0.5f * y, s0);
}
#endif

PBR_LX2_FN pbr_lv2 pbr_lx2_sel(int c0, int c1, pbr_lv2 a, pbr_lv2 b) {
    return (pbr_lv2){c0 ? a.x : b.x, c1 ? a.y : b.y};
}
PBR_LX2_FN pbr_lv2 pbr_lx2_abs(pbr_lv2 a) { return (pbr_lv2){PBR_LM_FABSF(a.x), PBR_LM_FABSF(a.y)}; }

/* s_atanf.c's reduction intervals as table rows {A, C, hi, lo}: the branch for |x| in [7/16, 11/16) computes
 * (2x - 1) / (x + 2), [11/16, 19/16) (x - 1) / (x + 1), [19/16, 39/16) (x - 1.5) / (1.5x + 1), [39/16, 2^25)
 * -1 / x, i.e. RN(RN(A x) - C) / RN(RN(C x) + A) with the row's A, C; row 4 (A = 1, C = 0: x / 1 = x, hi = lo = 0)
 * stands for |x| < 7/16 and, with its result replaced by the constant, for |x| >= 2^25. The device keeps the table
 * in LDS (pbr_device_math.h load_libm_tables): one 16-byte read per element instead of selects. */
typedef struct __attribute__((aligned(16))) {
    float a, c, hi, lo;
} pbr_atan_seg;
#define PBR_ATAN_SEG_TABLE_INIT                                          \
    {{2.0f, 1.0f, 4.6364760399e-01f, 5.0121582440e-09f},                \
     {1.0f, 1.0f, 7.8539812565e-01f, 3.7748947079e-08f},                \
     {1.0f, 1.5f, 9.8279368877e-01f, 3.4473217170e-08f},                \
     {0.0f, 1.0f, 1.5707962513e+00f, 7.5497894159e-08f},                \
     {1.0f, 0.0f, 0.0f, 0.0f}}

/* The table row for |x| (bit pattern ia, finite): 0..3 as above, 4 below 7/16 or at/above 2^25. */
PBR_LX2_FN int pbr_lx2_atan_row(uint32_t ia) {
    const int c = (ia >= 0x3ee00000u) + (ia >= 0x3f300000u) + (ia >= 0x3f980000u) + (ia >= 0x401c0000u) +
                  (ia >= 0x4c000000u);
    return c == 0 || c == 5 ? 4 : c - 1;
}

/* atanf(a) of s_atanf.c for a pair of finite a >= 0, branch-free. Division window: the denominators are 1, x + 2,
 * x + 1, 1.5x + 1 or x in [2.4375, 2^25) -- inside [1, 2^25]; the numerators 0, -1, multiples of 2^-24 of magnitude
 * <= 1, or x itself on row 4 (the caller keeps x == 0 or >= 2^-81). */
PBR_LX2_FN pbr_lv2 pbr_atanf_pos_x2(pbr_lv2 a, const pbr_atan_seg* tab) {
    PBR_LM_NO_CONTRACT
    const float a0 = 3.3333334327e-01f, a1 = -2.0000000298e-01f, a2 = 1.4285714924e-01f, a3 = -1.1111110449e-01f,
                a4 = 9.0908870101e-02f, a5 = -7.6918758452e-02f, a6 = 6.6610731184e-02f, a7 = -5.8335702866e-02f,
                a8 = 4.9768779427e-02f, a9 = -3.6531571299e-02f, a10 = 1.6285819933e-02f;
    const float huge = 1.5707962513e+00f + 7.5497894159e-08f; /* atanhi[3] + atanlo[3], rounded once */
    const uint32_t ia0 = pbr_lm_bits(a.x), ia1 = pbr_lm_bits(a.y);
    const pbr_atan_seg g0 = tab[pbr_lx2_atan_row(ia0)], g1 = tab[pbr_lx2_atan_row(ia1)];
    const pbr_lv2 A = {g0.a, g1.a}, C = {g0.c, g1.c};
    const pbr_lv2 x = pbr_lx2_div(A * a - C, C * a + A);
    const pbr_lv2 z = x * x;
    const pbr_lv2 w = z * z;
    const pbr_lv2 s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
    const pbr_lv2 s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
    const pbr_lv2 H = {g0.hi, g1.hi}, L = {g0.lo, g1.lo};
    const pbr_lv2 r = H - ((x * (s1 + s2) - L) - x);
    return pbr_lx2_sel(ia0 >= 0x4c000000u, ia1 >= 0x4c000000u, (pbr_lv2)(huge), r);
}

/* atan2f(y, x) of e_atan2f.c for a pair. special[e] = 1 where element e needs the scalar function: a NaN or
 * infinite component, or a nonzero magnitude outside [2^-40, 2^40]. Covered here: y == +-0, x == +-0, x == 1
 * (atanf(y) there: the same value through this path), |k| > 26 (the exponent-gap shortcuts), the quadrants. */
PBR_LX2_FN pbr_lv2 pbr_atan2f_x2(pbr_lv2 y, pbr_lv2 x, int special[2], const pbr_atan_seg* tab) {
    PBR_LM_NO_CONTRACT
    const float pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f, tiny = 1.0e-30f;
    const float big_z = pi_o_2 + 0.5f * pi_lo; /* k > 26 */
    const float c_pi = pi + tiny, c_npi = -pi - tiny, c_pio2 = pi_o_2 + tiny, c_npio2 = -pi_o_2 - tiny;
    const uint32_t hx[2] = {pbr_lm_bits(x.x), pbr_lm_bits(x.y)}, hy[2] = {pbr_lm_bits(y.x), pbr_lm_bits(y.y)};
    int m[2], kbig[2], kneg[2], yz[2], xz[2];
    for (int e = 0; e < 2; ++e) {
        const uint32_t ix = hx[e] & 0x7fffffffu, iy = hy[e] & 0x7fffffffu;
        const int in_x = ix == 0 || (ix >= 0x2b800000u && ix <= 0x53800000u); /* 0 or [2^-40, 2^40] */
        const int in_y = iy == 0 || (iy >= 0x2b800000u && iy <= 0x53800000u);
        special[e] = !(in_x && in_y);
        m[e] = (int)((hy[e] >> 31) & 1u) | (int)((hx[e] >> 30) & 2u);
        const int k = ((int)iy - (int)ix) >> 23;
        kbig[e] = k > PBR_ATAN2F_KMAX;
        kneg[e] = (hx[e] >> 31) && k < -PBR_ATAN2F_KMAX;
        yz[e] = iy == 0;
        xz[e] = ix == 0;
    }
    /* |y / x| in [2^-80, 2^80] when both are in [2^-40, 2^40]; lanes with a zero component divide 1 by 1. */
    const pbr_lv2 yy = pbr_lx2_sel(yz[0] | xz[0], yz[1] | xz[1], (pbr_lv2)(1.0f), y);
    const pbr_lv2 xx = pbr_lx2_sel(yz[0] | xz[0], yz[1] | xz[1], (pbr_lv2)(1.0f), x);
    pbr_lv2 z = pbr_atanf_pos_x2(pbr_lx2_abs(pbr_lx2_div(yy, xx)), tab);
    z = pbr_lx2_sel(kbig[0], kbig[1], (pbr_lv2)(big_z), z);
    z = pbr_lx2_sel(kneg[0], kneg[1], (pbr_lv2)(0.0f), z);
    const pbr_lv2 t = z - pi_lo;
    const pbr_lv2 q2 = pi - t, q3 = t - pi;
    pbr_lv2 r = pbr_lx2_sel(m[0] == 0, m[1] == 0, z, -z);
    r = pbr_lx2_sel(m[0] == 2, m[1] == 2, q2, r);
    r = pbr_lx2_sel(m[0] == 3, m[1] == 3, q3, r);
    /* y == +-0: y itself, +-pi by x's sign; then x == +-0: +-pi/2 by y's sign */
    const pbr_lv2 r_yz = pbr_lx2_sel(m[0] < 2, m[1] < 2, y, pbr_lx2_sel(m[0] == 2, m[1] == 2, (pbr_lv2)(c_pi),
                                                                         (pbr_lv2)(c_npi)));
    const pbr_lv2 r_xz = pbr_lx2_sel(hy[0] >> 31, hy[1] >> 31, (pbr_lv2)(c_npio2), (pbr_lv2)(c_pio2));
    r = pbr_lx2_sel(xz[0], xz[1], r_xz, r);
    return pbr_lx2_sel(yz[0], yz[1], r_yz, r);
}

/* asinf(x) of e_asinf.c for a pair, all three regimes evaluated and selected. special[e] = 1 for |x| > 1 or NaN
 * (the scalar function's (x - x) / (x - x)). Windows: below 0.5, no division; above, t = (1 - |x|) / 2 in
 * [2^-25, 0.25] (sqrt exponent >= -25), s + w in [2^-13, 1], t - w^2 exact-ish and >= 0 (0 or >= 2^-50). Lanes of
 * the other regime compute with harmless values (t in (0.25, 0.5] below 0.5; |x| == 1 selects its own result). */
PBR_LX2_FN pbr_lv2 pbr_asinf_x2(pbr_lv2 x, int special[2]) {
    PBR_LM_NO_CONTRACT
    const float pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
                pio4_hi = 0.785398185253143310546875f;
    const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                p4 = 4.216630880e-2f;
    const uint32_t hx[2] = {pbr_lm_bits(x.x), pbr_lm_bits(x.y)};
    const uint32_t ix[2] = {hx[0] & 0x7fffffffu, hx[1] & 0x7fffffffu};
    special[0] = ix[0] > 0x3f800000u;
    special[1] = ix[1] > 0x3f800000u;
    /* |x| < 0.5 (below 2^-27 this is x itself, as the scalar function's early return) */
    const pbr_lv2 ts = x * x;
    const pbr_lv2 ws = ts * (p0 + ts * (p1 + ts * (p2 + ts * (p3 + ts * p4))));
    const pbr_lv2 r_small = x + x * ws;
    /* |x| >= 0.5 (|x| == 1 takes its own formula below) */
    const int one0 = ix[0] == 0x3f800000u, one1 = ix[1] == 0x3f800000u;
    const pbr_lv2 ax = pbr_lx2_sel(one0, one1, (pbr_lv2)(0.5f), pbr_lx2_abs(x));
    const pbr_lv2 wl = 1.0f - ax;
    const pbr_lv2 t = wl * 0.5f;
    const pbr_lv2 p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    const pbr_lv2 s = pbr_lx2_sqrt(t);
    const pbr_lv2 r_far = pio2_hi - (2.0f * (s + s * p) - pio2_lo); /* |x| >= 0.975 */
    const pbr_lv2 w = (pbr_lv2){pbr_lm_float(pbr_lm_bits(s.x) & 0xfffff000u), pbr_lm_float(pbr_lm_bits(s.y) & 0xfffff000u)};
    const pbr_lv2 c = pbr_lx2_div(t - w * w, s + w);
    const pbr_lv2 pp = 2.0f * s * p - (pio2_lo - 2.0f * c);
    const pbr_lv2 q = pio4_hi - 2.0f * w;
    const pbr_lv2 r_mid = pio4_hi - (pp - q);
    pbr_lv2 r = pbr_lx2_sel(ix[0] >= 0x3f79999au, ix[1] >= 0x3f79999au, r_far, r_mid);
    r = pbr_lx2_sel(hx[0] >> 31, hx[1] >> 31, -r, r);
    r = pbr_lx2_sel(ix[0] < 0x3f000000u, ix[1] < 0x3f000000u, r_small, r);
    const pbr_lv2 r_one = x * pio2_hi + x * pio2_lo;
    return pbr_lx2_sel(one0, one1, r_one, r);
}

#endif /* PBR_LIBM_F32_X2_H */
