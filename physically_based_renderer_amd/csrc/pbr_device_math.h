// pbr_device_math.h -- gfx950 device-side restatement of the reference BRDF
// (Source/Shaders/LightingUtil.hlsl:35-225) in HLSL fp32 semantics.
//
// Parity with the CPU evaluation needs op-for-op identical fp32 arithmetic ("canonical
// fp32 semantics"): this file is compiled with -ffp-contract=off and correctly rounded fp32
// division/sqrt (-fhip-fp32-correctly-rounded-divide-sqrt), never -ffast-math. Every expression
// below keeps the reference's evaluation order; the only rewrites are hoists of per-pixel
// invariants out of the light loop, which compute the identical values once instead of per light.
#pragma once
#include <hip/hip_runtime.h>
#include "libm_f32.h"
#include "libm_f32_x2.h"
#include "pbr_debug_bounds.h"
#include "pbr_census.h"

namespace pbr {

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add3(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
// HLSL dot: (a.x*b.x + a.y*b.y) + a.z*b.z, no fused multiply-add.
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// HLSL max / saturate on D3D10+: IEEE maxNum (NaN operand -> the other one), saturate(NaN) = 0.
__device__ __forceinline__ float hmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ float hsat(float a) { return fminf(fmaxf(a, 0.0f), 1.0f); }
// normalize(v) = v / sqrt(dot(v, v)): three IEEE divides, not v * rsqrt.
__device__ __forceinline__ f3 normalize3(f3 v) {
    float s = sqrtf(dot3(v, v));
    return mk3(v.x / s, v.y / s, v.z / s);
}
__device__ __forceinline__ float hlerp(float x, float y, float s) { return x + s * (y - x); }

// ---- Exact fast paths --------------------------------------------------------------------------
// With correctly rounded division, hipcc expands each x / y into ~11 operations (v_div_scale x2,
// v_rcp, two Newton fma, three correction fma/mul, v_div_fmas, v_div_fixup) plus hazard NOPs; the
// scale and fix-up steps exist for operands near the ends of the exponent range, zeros, infinities
// and NaNs. Inside a window that excludes those cases the quotient is computed here as:
//   y = recip_nr(b):  r = v_rcp(b); e = fma(-b, r, 1); y = fma(e, r, r)
//       -- equals RN(1/b), the correctly rounded reciprocal, for EVERY significand at every exponent
//          in [-64, 64] (exhaustive check on gfx950: tests/test_gpu_fastdiv.py);
//   q = div_nr(a, y): q0 = a*y; t = fma(b, q0, -a); q = fma(-t, y, q0)
//       -- Markstein's theorem: with y = RN(1/b), q0 within one ulp of a/b and the residual exact
//          (fma), RN(q0 + (a - b q0) y) = RN(a/b). t is formed as -(a - b q0) so that a -0
//          numerator keeps its sign for b > 0 (the plain form returns +0 there).
// Window (proved per pixel-light by the callers, see fast_window_ok): 0 < b in [2^-60, 2^60];
// a == +-0 or |a| in [2^-96, 2^60]; |a / b| in [2^-120, 2^120] (no overflow, no subnormal q0 or t).
// One reciprocal serves every numerator with the same denominator (L/d, normalize, specular, /PI).
// The light loop falls back to the compiler's full sequences whenever the window is not proved;
// PBR_FLAG_EXACT_ONLY runs only those, and tests require both modes to agree bit for bit
// (tests/test_gpu_parity.py::test_fast_path_is_bit_identical_to_exact_only).
struct Recip {
    float y, r;
};
__device__ __forceinline__ Recip recip_nr(float y) {
    float r = __builtin_amdgcn_rcpf(y);
    float e = __builtin_fmaf(-y, r, 1.0f);
    return Recip{y, __builtin_fmaf(e, r, r)};
}
__device__ __forceinline__ float div_nr(float x, Recip d) {
    float q = x * d.r;
    float t = __builtin_fmaf(d.y, q, -x);
    return __builtin_fmaf(-t, d.r, q);
}
// sqrt in five operations: y = v_rsq(x), s0 = x*y, r = x - s0^2 (fma), s = s0 + r*(y/2) (fma). Probed
// on gfx950 to equal the IEEE sqrtf for every float with exponent in [-64, 64] (tests/hip/sqrt_probe.hip,
// test_gpu_probes.py); the window checks keep every use inside that range (dist >= 2^-20, |V+L| >= 2^-30;
// x = 0 gives NaN, which fails them).
__device__ __forceinline__ float sqrt_nr(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y;
    const float r = __builtin_fmaf(-s0, s0, x);
    return __builtin_fmaf(r, 0.5f * y, s0);
}
// |x| in [lo, hi] (false for NaN); zero_or_in also accepts +-0.
__device__ __forceinline__ bool in_win(float x, float lo, float hi) { return fabsf(x) >= lo && fabsf(x) <= hi; }
__device__ __forceinline__ bool zero_or_in(float x, float lo, float hi) { return x == 0.0f || in_win(x, lo, hi); }

// pow(x, 5.0) of FresnelSchlick (LightingUtil.hlsl:46) for x = 1 - saturate(.) in {0} U [2^-24, 1].
//
// The oracle computes glibc's powf, which is 1 ulp off the correctly rounded x^5 on 0.06% of
// inputs. Where that matters is kD = 1 - F: with p = x^5, one ulp of p becomes p / (1 - p) ulps of kD.
//  * pow5_glibc: glibc's algorithm bit for bit (libm_f32.h). Used for the IBL ambient's Fresnel
//    (Default.hlsl:141-146; once per pixel, and there kD scales the whole term), and by pow5_light
//    on the grazing band.
//  * pow5_light: per light, fp64 x^5 (2^-52 relative before the one rounding to fp32; correctly
//    rounded on every float in [0, 1] checked) while x <= 0.99, glibc's algorithm above. On the fp64
//    side p <= 0.951, so a 1-ulp difference from glibc moves that light's diffuse term by at most
//    19.4 ulp (1.2e-6 relative) and leaves every other term exact -- 8x inside the 1e-5 parity bar
//    even for a pixel lit by that light alone. x > 0.99 needs H.V < 0.01 and is rare per wave.
// The tables are read from LDS (PBR_POW5_LDS, filled by load_libm_tables at kernel entry) or from
// constant memory.
#ifndef PBR_POW5_LDS
#define PBR_POW5_LDS 1
#endif
#if PBR_POW5_LDS
// The three tables back to back, 37 chunks of 16 bytes: powf's log2 rows (16 x 16 B), its exp2 words (32 x 8 B),
// atanf's reduction rows (5 x 16 B). load_libm_tables copies them with one 16-byte load per work-item and a single
// wait (three separately predicated copies each waited for their own load: three round trips before a wave's
// G-buffer loads could issue).
struct alignas(16) LibmTables {
    pbr_powf_log2_entry log2[16];
    uint64_t exp2[32];
    pbr_atan_seg atan[5];  // libm_f32_x2.h
};
static_assert(sizeof(LibmTables) == 37 * 16, "one 16-byte chunk per work-item");
__shared__ LibmTables g_lds_libm;
static __constant__ LibmTables pbr_libm_tables = {PBR_POWF_LOG2_TABLE_INIT, PBR_EXP2F_TABLE_INIT,
                                                  PBR_ATAN_SEG_TABLE_INIT};
// Every work-item of the block calls this, and a barrier follows before the first table read. ATAN: the kernel
// evaluates the packed WorldToSkyUV (diffuse-IBL ambient); otherwise the atan rows are not copied.
template <bool ATAN = true>
__device__ __forceinline__ void load_libm_tables() {
    constexpr int kChunks = ATAN ? 37 : 32;
    const int t = threadIdx.x;
    if (t < kChunks) reinterpret_cast<uint4*>(&g_lds_libm)[t] = reinterpret_cast<const uint4*>(&pbr_libm_tables)[t];
}
#define PBR_POW5_TABLES g_lds_libm.log2, g_lds_libm.exp2
#define PBR_LIBM_LOG2_TAB g_lds_libm.log2
#define PBR_LIBM_EXP2_TAB g_lds_libm.exp2
#define PBR_LIBM_ATAN_TAB g_lds_libm.atan
#else
static __constant__ pbr_atan_seg pbr_atan_seg_tab[5] = PBR_ATAN_SEG_TABLE_INIT;
template <bool ATAN = true>
__device__ __forceinline__ void load_libm_tables() {}
#define PBR_POW5_TABLES pbr_powf_log2_tab, pbr_exp2f_tab
#define PBR_LIBM_LOG2_TAB pbr_powf_log2_tab
#define PBR_LIBM_EXP2_TAB pbr_exp2f_tab
#define PBR_LIBM_ATAN_TAB pbr_atan_seg_tab
#endif
#ifndef PBR_POW5_GLIBC_FROM  // x above which pow5_light switches to glibc's algorithm
#define PBR_POW5_GLIBC_FROM 0.99f
#endif
__device__ __forceinline__ float pow5_glibc(float x) { return pbr_pow5_unit(x, PBR_POW5_TABLES); }
__device__ __forceinline__ float pow5_light(float x) {
    if (__builtin_expect(x > PBR_POW5_GLIBC_FROM, 0)) return pow5_glibc(x);
    const double d = (double)x;
    const double d2 = d * d;
    return (float)(d2 * d2 * d);
}
// powf for the spot cone and the gamma encode: glibc's algorithm (libm_f32.h), all special cases.
__device__ __forceinline__ float powf_glibc(float x, float y) { return pbr_powf(x, y); }

constexpr float kPi = 3.14159265359f;  // LightingUtil.hlsl:59, 103 (an fp32 literal in HLSL)

// x / kPi in two operations: q = fma(x, zh, x * zl) with zh = RN(1/kPi), zl = RN(1/kPi - zh). Checked
// exhaustively to equal the IEEE quotient for every significand (tests: test_div_pi_is_exact on the
// host, fastdiv_probe on the GPU), hence for every |x| in [2^-98, 2^100] or 0, where x * zl stays
// normal. In the fast-path window kD * albedo is 0 or >= 2^-68 in magnitude (|1-F|, 1-metallic >= 2^-24
// or 0; albedo >= 2^-20).
constexpr float kInvPiHi = 0x1.45f306p-2f, kInvPiLo = 0x1.11be6cp-28f;
__device__ __forceinline__ float div_pi(float x) { return __builtin_fmaf(x, kInvPiHi, x * kInvPiLo); }
constexpr float kInvGamma = 1.0f / 2.2f;  // Default.hlsl:155

// pow(c, 1/2.2) of the gamma step (Default.hlsl:155, Skybox.hlsl:48) as glibc's powf: for c in
// [2^-126, 1) -- every tonemapped value of a finite non-negative colour but 0 -- none of powf's special
// cases apply and |y log2 c| < 58 cannot overflow, so its main path runs directly on the LDS tables;
// anything else takes the general function.
__device__ __forceinline__ float pow_inv_gamma(float c) {
    const uint32_t ix = __float_as_uint(c);
    if (__builtin_expect(ix - 0x00800000u < 0x3f800000u - 0x00800000u, 1))
        return pbr_powf_exp2((double)kInvGamma * pbr_powf_log2(ix, PBR_LIBM_LOG2_TAB), 0u, PBR_LIBM_EXP2_TAB);
    return pbr_powf(c, kInvGamma);
}
// PBR_FLAG_FAITHFUL's gamma encode: exp2(kInvGamma * log2(c)) on the hardware v_log_f32 / v_exp_f32
// for c in [kFaithfulGammaLo, 1) and for c = +-0 (log2 gives -inf, exp2 +0: powf's own +0), glibc's powf
// elsewhere. Error vs glibc powf measured exhaustively on the GPU per binade (tests/hip/gamma_probe.hip,
// profiles/r04/gamma_window_scan.log): <= 5.4e-7 from 2^-10 up, <= 1.04e-6 down to 2^-32, 1.6-2.0e-6 below
// (the rounding of kInvGamma * log2(c) grows with |log2 c|), hence the window's 2^-32; DESIGN.md §2 adds
// 1.04e-6 to the faithful bound. (Round 3's window began at 2^-10, which sent nearly every wave of configs 2
// and 3 through glibc's algorithm for some dark channel.)
#ifndef PBR_FAITHFUL_GAMMA_LO
#define PBR_FAITHFUL_GAMMA_LO 0x1p-32f
#endif
constexpr float kFaithfulGammaLo = PBR_FAITHFUL_GAMMA_LO;
__device__ __forceinline__ float pow_inv_gamma_faithful(float c) {
    if (__builtin_expect((c >= kFaithfulGammaLo && c < 1.0f) || c == 0.0f, 1))
        return __builtin_amdgcn_exp2f(kInvGamma * __builtin_amdgcn_logf(c));
    return pow_inv_gamma(c);
}
constexpr float kLightRange = 100.0f;     // LightingUtil.hlsl:131

// Everything BRDFCookTorrance (LightingUtil.hlsl:85-104) needs that does not depend on the light.
struct PixelInvariants {
    f3 n, v, albedo, f0;
    f3 one_minus_f0;      // (1.0f - F0) of FresnelSchlick (:46)
    float one_minus_metal;  // 1.0f - mat.Metallic (:100)
    float a_sqr;            // DistributionGGX: r = max(rough, 0.05), a = r*r, aSqr = a*a (:51-53)
    float a_sqr_minus_1;    // (aSqr - 1.0f) (:58)
    float k, one_minus_k;   // GeometrySchlickGGX: k = (r+1)^2 / 8 on the unclamped roughness (:66-67)
    float ggx_v;            // GeometrySchlickGGX(NdotV) = ggx2 (:79)
    float four_n_dot_v;     // 4.0f * max(dot(N,V), 0) (:95, left operand of the product)
    bool fast_ok;           // the pixel's inputs lie in the fast-path window (see below)
    bool f0_nonzero;        // no F0 component is zero
};

// Per-pixel half of the fast-path proof ("exact fast path"). With every position
// component (pixel and eye) zero or of magnitude [2^-20, 2^20], normal components zero or
// [2^-20, 16], albedo/F0 components zero or [2^-20, 1024], metallic and roughness in [0, 1]:
//   L = lightPos - P has components 0 or [2^-43, 2^21]; V and L/d components 0 or >= 2^-65;
//   (V + L) components 0 or >= 2^-88; N.L is 0 or >= 2^-93; GeometrySchlickGGX's denominator is
//   in [0.125, 48.5]; kD*albedo is 0 or in [2^-68, 2^21].
// Together with the per-iteration compares in the light functions this keeps every fast-path
// division and sqrt inside the windows stated above.
// The per-pixel window as unsigned min/max over bit patterns (no compare-and-branch chains): a value
// passes "0 or |x| in [2^-20, hi]" iff b = bits(|x|) satisfies b - 1 >= bits(2^-20) - 1 (unsigned:
// b = 0 wraps to the maximum) and b <= bits(hi); NaN and inf exceed every hi. Metallic and roughness
// must lie in [0, 1] (or be -0). The eye position (uniform) is checked once on the host (PassArgs).
__device__ __forceinline__ uint32_t abs_bits(float x) { return __float_as_uint(x) & 0x7fffffffu; }
__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) { return min(min(a, b), c); }
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) { return max(max(a, b), c); }
__device__ __forceinline__ bool unit_or_neg_zero(float x) {
    const uint32_t b = __float_as_uint(x);
    return b <= 0x3f800000u || b == 0x80000000u;
}
__device__ __forceinline__ bool fast_window_ok(f3 pos, f3 n, f3 albedo, f3 f0, float metallic, float roughness) {
    const uint32_t bp[3] = {abs_bits(pos.x), abs_bits(pos.y), abs_bits(pos.z)};
    const uint32_t bn[3] = {abs_bits(n.x), abs_bits(n.y), abs_bits(n.z)};
    const uint32_t ba[3] = {abs_bits(albedo.x), abs_bits(albedo.y), abs_bits(albedo.z)};
    const uint32_t bf[3] = {abs_bits(f0.x), abs_bits(f0.y), abs_bits(f0.z)};
    const uint32_t lo = umin3(umin3(bp[0] - 1u, bp[1] - 1u, bp[2] - 1u), umin3(bn[0] - 1u, bn[1] - 1u, bn[2] - 1u),
                              min(umin3(ba[0] - 1u, ba[1] - 1u, ba[2] - 1u), umin3(bf[0] - 1u, bf[1] - 1u, bf[2] - 1u)));
    const bool lo_ok = lo >= 0x35800000u - 1u;                          // 2^-20
    const bool pos_ok = umax3(bp[0], bp[1], bp[2]) <= 0x49800000u;      // 2^20
    const bool n_ok = umax3(bn[0], bn[1], bn[2]) <= 0x41800000u;        // 16
    const bool af_ok = max(umax3(ba[0], ba[1], ba[2]), umax3(bf[0], bf[1], bf[2])) <= 0x44800000u;  // 1024
    return ((int)lo_ok & (int)pos_ok & (int)n_ok & (int)af_ok & (int)unit_or_neg_zero(metallic) &
            (int)unit_or_neg_zero(roughness)) != 0;
}

// F0 with no zero component: then F = F0 + (1-F0) p stays >= 2^-20 for any p (see brdf checks).
__device__ __forceinline__ bool f0_nonzero(f3 f0) { return f0.x != 0.0f && f0.y != 0.0f && f0.z != 0.0f; }

// Per-light half, evaluated once when the light is staged: point/spot positions like pixel
// positions; directional L = -Direction components zero or [2^-20, 16].
__device__ __forceinline__ bool light_window_ok(bool directional, float4 dir, float4 pos) {
    const float lo = 0x1p-20f;
    if (directional)
        return zero_or_in(dir.x, lo, 16.0f) && zero_or_in(dir.y, lo, 16.0f) && zero_or_in(dir.z, lo, 16.0f);
    return zero_or_in(pos.x, lo, 0x1p20f) && zero_or_in(pos.y, lo, 0x1p20f) && zero_or_in(pos.z, lo, 0x1p20f);
}

__device__ __forceinline__ PixelInvariants make_invariants(f3 n, f3 v, f3 albedo, f3 f0, float metallic,
                                                           float roughness) {
    PixelInvariants q;
    q.n = n;
    q.v = v;
    q.albedo = albedo;
    q.f0 = f0;
    q.one_minus_f0 = mk3(1.0f - f0.x, 1.0f - f0.y, 1.0f - f0.z);
    q.one_minus_metal = 1.0f - metallic;
    float r = hmax(roughness, 0.05f);
    float a = r * r;
    q.a_sqr = a * a;
    q.a_sqr_minus_1 = q.a_sqr - 1.0f;
    float rr = (roughness + 1.0f);
    q.k = (rr * rr) / 8.0f;
    q.one_minus_k = 1.0f - q.k;
    float n_dot_v = hmax(dot3(n, v), 0.0f);
    q.ggx_v = n_dot_v / (n_dot_v * q.one_minus_k + q.k);
    q.four_n_dot_v = 4.0f * n_dot_v;
    q.fast_ok = false;
    q.f0_nonzero = f0_nonzero(f0);
    return q;
}

// x / d.y either through the exact fast sequence (FAST) or the compiler's full IEEE division.
template <bool FAST>
__device__ __forceinline__ float qdiv(float x, Recip d) {
    return FAST ? div_nr(x, d) : x / d.y;
}
template <bool FAST>
__device__ __forceinline__ Recip qrecip(float y) {
    return FAST ? recip_nr(y) : Recip{y, 0.0f};
}

// BRDFCookTorrance (LightingUtil.hlsl:85-104) with DistributionGGX (:49-62), GeometrySmith (:75-83)
// and FresnelSchlick (:43-47) inlined; returns (kD*albedo/PI + specular) * radiance * NdotL.
// FAST: ANDs into `ok` the window conditions the pixel/light flags cannot guarantee.
template <bool FAST>
__device__ __forceinline__ f3 brdf_cook_torrance(const PixelInvariants& q, f3 radiance, f3 l, f3 h, bool& ok) {
    // DistributionGGX
    float n_dot_h = hmax(dot3(q.n, h), 0.0f);
    float n_dot_h_sqr = n_dot_h * n_dot_h;
    float den = (n_dot_h_sqr * q.a_sqr_minus_1 + 1.0f);
    den = kPi * den * den;
    if (FAST) ok = ok && den >= 0x1p-60f && den <= 0x1p60f;
    float ndf = qdiv<FAST>(q.a_sqr, qrecip<FAST>(den));
    // GeometrySmith: ggx1 * ggx2
    float n_dot_l = hmax(dot3(q.n, l), 0.0f);
    float ggx_l = qdiv<FAST>(n_dot_l, qrecip<FAST>(n_dot_l * q.one_minus_k + q.k));
    float g = ggx_l * q.ggx_v;
    // FresnelSchlick(H, V, F0)
    float cos_theta = hsat(dot3(h, q.v));
    float p = pow5_light(1.0f - cos_theta);
    f3 f = mk3(q.f0.x + q.one_minus_f0.x * p, q.f0.y + q.one_minus_f0.y * p, q.f0.z + q.one_minus_f0.z * p);
    // specular = (NDF*G)*F / (4*NdotV*NdotL + 0.001); the denominator is >= 0.001 by construction
    float ndf_g = ndf * g;
    float denom = q.four_n_dot_v * n_dot_l + 0.001f;
    f3 nom = mk3(ndf_g * f.x, ndf_g * f.y, ndf_g * f.z);
    if (FAST) {
        // F components are 0 or in [2^-40, 2^11] (F0 window; p == 0 or >= 2^-40 unless F0 has no
        // zero), so nom = NDF*G*F is 0 or in [2^-70, 2^51] when NDF*G is 0 or in [2^-30, 2^40];
        // denom is in [0.001, 2^17] by the pixel and light windows.
        ok = ok && zero_or_in(ndf_g, 0x1p-30f, 0x1p40f) && (q.f0_nonzero || p == 0.0f || p >= 0x1p-40f);
    }
    const Recip rdenom = qrecip<FAST>(denom);
    f3 spec = mk3(qdiv<FAST>(nom.x, rdenom), qdiv<FAST>(nom.y, rdenom), qdiv<FAST>(nom.z, rdenom));
    // kD = (1 - F) * (1 - metallic)
    f3 kd = mk3((1.0f - f.x) * q.one_minus_metal, (1.0f - f.y) * q.one_minus_metal, (1.0f - f.z) * q.one_minus_metal);
    const f3 kda = mk3(kd.x * q.albedo.x, kd.y * q.albedo.y, kd.z * q.albedo.z);
    const f3 diffuse = FAST ? mk3(div_pi(kda.x), div_pi(kda.y), div_pi(kda.z))
                            : mk3(kda.x / kPi, kda.y / kPi, kda.z / kPi);
    return mk3(((diffuse.x + spec.x) * radiance.x) * n_dot_l, ((diffuse.y + spec.y) * radiance.y) * n_dot_l,
               ((diffuse.z + spec.z) * radiance.z) * n_dot_l);
}

// normalize(v) through the fast path: sqrt_nr + three divisions sharing one refined reciprocal.
template <bool FAST>
__device__ __forceinline__ f3 normalize_q(f3 v, bool& ok) {
    if (!FAST) return normalize3(v);
    float s = sqrt_nr(dot3(v, v));
    ok = ok && s >= 0x1p-30f;  // s <= 1 + |L| <= 29 by the windows
    const Recip r = recip_nr(s);
    return mk3(div_nr(v.x, r), div_nr(v.y, r), div_nr(v.z, r));
}

// ComputeDirectionalLight (LightingUtil.hlsl:109-119). The caller adds shadowFactor(1,1,1) * result,
// and 1.0f * x == x exactly, so the multiply is omitted.
template <bool FAST>
__device__ __forceinline__ f3 directional_light(const PixelInvariants& q, float4 s, float4 d, bool& ok) {
    f3 l = mk3(-d.x, -d.y, -d.z);
    f3 h = normalize_q<FAST>(add3(q.v, l), ok);
    return brdf_cook_torrance<FAST>(q, mk3(s.x, s.y, s.z), l, h, ok);
}

// ComputePointLight (:124-142) / ComputeSpotLight (:147-167). Returns false when the range test at
// :131 / :154 returns 0: adding +0 to the running sum is the identity (the sum starts at +0 and is
// never -0), so skipping it is bit-exact. The range decision is exact on the fast path too: sqrt_nr
// is exact on [2^-96, 2^128) and gives 0 / inf / NaN outside, all on the same side of 100.
template <bool SPOT, bool FAST>
__device__ __forceinline__ bool point_or_spot_light(const PixelInvariants& q, f3 pos, float4 s, float4 d, float4 p,
                                                    f3& out, bool& ok) {
    f3 l = mk3(p.x - pos.x, p.y - pos.y, p.z - pos.z);
    float dist = FAST ? sqrt_nr(dot3(l, l)) : sqrtf(dot3(l, l));
    if (dist > kLightRange) return false;
    if (FAST) ok = ok && dist >= 0x1p-20f;
    const Recip rdist = qrecip<FAST>(dist);
    l = mk3(qdiv<FAST>(l.x, rdist), qdiv<FAST>(l.y, rdist), qdiv<FAST>(l.z, rdist));
    f3 h = normalize_q<FAST>(add3(q.v, l), ok);
    float dsat = hmax(dist, 0.01f);  // CalcAttenuation (:35-40); dsat^2 in [1e-4, 1e4]
    // 1 / dsat^2: the refined reciprocal is already RN(1/y) in this window (exponents [-14, 14])
    float att = FAST ? qrecip<FAST>(dsat * dsat).r : 1.0f / (dsat * dsat);
    if (SPOT) {
        f3 nl = mk3(-l.x, -l.y, -l.z);
        att *= powf_glibc(hmax(dot3(nl, mk3(d.x, d.y, d.z)), 0.0f), s.w);  // :163, SpotPower in .w
    }
    out = brdf_cook_torrance<FAST>(q, mk3(s.x * att, s.y * att, s.z * att), l, h, ok);
    return true;
}

// WorldToSkyUV (LightingUtil.hlsl:216-225); .xy only.
__device__ __forceinline__ void world_to_sky_uv(f3 c, float& u, float& v) {
    float ux = pbr_atan2f(c.z, c.x);  // glibc's algorithms, bit for bit (libm_f32.h)
    float uy = pbr_asinf(c.y);
    ux = ux * 0.1591f;
    uy = uy * 0.3183f;
    ux = ux + 0.5f;
    uy = uy + 0.5f;
    uy = 1.0f - uy;
    ux = 1.0f - ux;
    ux = ux + 0.25f;
    u = ux;
    v = uy;
}

__device__ __forceinline__ int wrap_index(float f, int n) {
    if (!(f == f) || f > 2.0e9f || f < -2.0e9f) return 0;  // NaN coordinate: the weights are NaN anyway
    const int i = (int)f;
    if (__builtin_expect(i >= -n && i < 2 * n, 1)) {  // every finite WorldToSkyUV texel: one wrap at most
        const int j = i < 0 ? i + n : i;
        return j >= n ? j - n : j;                     // == ((i % n) + n) % n on this range
    }
    PBR_COLD("wrap_mod");
    const int m = i % n;
    return m < 0 ? m + n : m;
}

// Linear-wrap bilinear sample (g_SamLinearWrap, PBRApp.cpp:1157-1162) of the fp32 RGBA env map
// (texels pre-decoded as u16 / 65535.0f), in the fp32 formula fixed by DESIGN.md.
__device__ __forceinline__ f3 sample_linear_wrap(const float4* __restrict__ env, int w, int h, float u, float v) {
    float x = u * (float)w - 0.5f;
    float y = v * (float)h - 0.5f;
    float x0f = floorf(x), y0f = floorf(y);
    float fx = x - x0f, fy = y - y0f;
    int x0 = wrap_index(x0f, w), y0 = wrap_index(y0f, h);
    int x1 = x0 + 1 == w ? 0 : x0 + 1;
    int y1 = y0 + 1 == h ? 0 : y0 + 1;
    [[maybe_unused]] const int64_t n = (int64_t)w * h;
    float4 t00 = env[PBR_BOUNDS(y0 * w + x0, n, kBoundsTexel)], t10 = env[PBR_BOUNDS(y0 * w + x1, n, kBoundsTexel)];
    float4 t01 = env[PBR_BOUNDS(y1 * w + x0, n, kBoundsTexel)], t11 = env[PBR_BOUNDS(y1 * w + x1, n, kBoundsTexel)];
    return mk3(hlerp(hlerp(t00.x, t10.x, fx), hlerp(t01.x, t11.x, fx), fy),
               hlerp(hlerp(t00.y, t10.y, fx), hlerp(t01.y, t11.y, fx), fy),
               hlerp(hlerp(t00.z, t10.z, fx), hlerp(t01.z, t11.z, fx), fy));
}

}  // namespace pbr
