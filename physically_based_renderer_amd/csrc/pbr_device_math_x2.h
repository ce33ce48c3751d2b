// pbr_device_math_x2.h -- the exact fast path of pbr_device_math.h for a PAIR of pixels per
// work-item, in packed fp32 (gfx950 v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32).
//
// Every operation is the scalar fast path's operation applied element-wise: a packed instruction
// rounds each element exactly like its scalar form, so each pixel of the pair gets the bits the
// scalar fast path (and therefore the compiler's full IEEE sequences) would give it. Transcendental
// seeds (v_rcp_f32, v_rsq_f32), compares, selects and the fp64 powf (pow5) have no packed form and run
// per element. Pixels that leave the fast-path window are re-evaluated by the scalar exact path.
#pragma once
#include <cstdint>

#include "pbr_device_math.h"

namespace pbr {

typedef float v2 __attribute__((ext_vector_type(2)));

// Per-element conditions of the pair as wave lane masks (bit l = work-item l of the wave): a compare
// writes its mask straight into an SGPR pair, and combining masks (the fast-path window, the redo
// set) runs on the scalar unit instead of as v_cndmask / v_and / v_or on VGPR int vectors. Every
// function below that builds or reads a mask is called by all lanes of the wave (uniform control flow).
struct m2 {
    uint64_t x, y;
};
__device__ __forceinline__ uint64_t lanes(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ bool on(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ m2 operator&(m2 a, m2 b) { return m2{a.x & b.x, a.y & b.y}; }
__device__ __forceinline__ m2 operator|(m2 a, m2 b) { return m2{a.x | b.x, a.y | b.y}; }
__device__ __forceinline__ m2 operator~(m2 a) { return m2{~a.x, ~a.y}; }
__device__ __forceinline__ m2& operator&=(m2& a, m2 b) { return a = a & b; }
__device__ __forceinline__ m2& operator|=(m2& a, m2 b) { return a = a | b; }
__device__ __forceinline__ m2 mask2(bool x, bool y) { return m2{lanes(x), lanes(y)}; }
__device__ __forceinline__ m2 all2(bool c) { const uint64_t m = lanes(c); return m2{m, m}; }

// ---- Wave-wide reductions and scans on the DPP network (no LDS round trips) ----
// __shfl_xor / __shfl_up compile to ds_bpermute: each step an LDS round trip (and its address arithmetic), six in a
// row per reduction. Here the first four steps are DPP lane moves fused into the combining instruction (quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: every lane of a 16-lane row then holds the row's result), and
// the rows meet on the scalar unit (v_readlane of lanes 0, 16, 32, 48). Min / max run on an integer key whose signed
// order is the float order (non-NaN floats; -0 below +0, which changes no value computed from the result); a NaN
// input counts as `neutral` (fminf / fmaxf also ignore a NaN operand). The result is wave-uniform (SGPR).
template <int CTRL>
__device__ __forceinline__ int dpp_row_move(int v) {  // sources always inside the row: bound_ctrl lets it fuse
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ int float_key(float f) {
    const int b = __builtin_bit_cast(int, f);
    return b ^ (int)((uint32_t)(b >> 31) >> 1);
}
__device__ __forceinline__ float key_float(int k) { return __builtin_bit_cast(float, k ^ (int)((uint32_t)(k >> 31) >> 1)); }
template <bool MAX>
__device__ __forceinline__ float wave_minmax_dpp(float v, float neutral) {
    int k = float_key(v == v ? v : neutral);
    auto op = [](int a, int b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    k = op(k, dpp_row_move<0xB1>(k));   // quad_perm [1,0,3,2]
    k = op(k, dpp_row_move<0x4E>(k));   // quad_perm [2,3,0,1]
    k = op(k, dpp_row_move<0x141>(k));  // row_half_mirror
    k = op(k, dpp_row_move<0x140>(k));  // row_mirror
    const int r = op(op(__builtin_amdgcn_readlane(k, 0), __builtin_amdgcn_readlane(k, 16)),
                     op(__builtin_amdgcn_readlane(k, 32), __builtin_amdgcn_readlane(k, 48)));
    return key_float(r);
}
__device__ __forceinline__ float wave_min_dpp(float v, float neutral = 3.0e38f) { return wave_minmax_dpp<false>(v, neutral); }
__device__ __forceinline__ float wave_max_dpp(float v, float neutral = -3.0e38f) { return wave_minmax_dpp<true>(v, neutral); }
// Min / max over the wave of FINITE floats (the balanced pass-1 box of a fast-window wave: every position and bound is
// finite there), on the float unit: v_min_f32_dpp / v_max_f32_dpp through the four in-row steps, then row_bcast 15 / 31
// carry the row results up (rows 1, 3, then 2, 3), so lane 63 holds the wave's result: one v_readlane. No order key, no
// NaN mapping, no scalar combine of four row results (which needed VGPR moves for its three-operand form): 6 DPP
// instructions and a readlane instead of ~17 VALU. Inline asm with the two wait states a DPP read of a VGPR written by
// the previous VALU instruction needs (s_nop 1); every lane must be active. -0 and +0 may come out either way (IEEE
// minNum), which changes nothing computed from a bound.
template <bool MAX>
__device__ __forceinline__ float wave_minmax_finite(float v) {
    if constexpr (MAX) {
        asm volatile(
            "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
            "s_nop 1"
            : "+v"(v));
    } else {
        asm volatile(
            "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
            "s_nop 1"
            : "+v"(v));
    }
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ float wave_min_finite(float v) { return wave_minmax_finite<false>(v); }
__device__ __forceinline__ float wave_max_finite(float v) { return wave_minmax_finite<true>(v); }
// fminf / fmaxf of finite operands as one instruction (the compiler quiets operands it cannot prove canonical with an
// extra v_max each, as IEEE mode requires for a possible signalling NaN; none reaches these).
__device__ __forceinline__ float fmin_finite(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float fmax_finite(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// Sum over the wave, wave-uniform.
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += dpp_row_move<0xB1>(v);
    v += dpp_row_move<0x4E>(v);
    v += dpp_row_move<0x141>(v);
    v += dpp_row_move<0x140>(v);
    return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
           (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
}
// Inclusive prefix sum over the lanes: row_shr 1, 2, 4, 8 within each row (lanes shifted in from outside it read 0),
// then row_bcast 15 / 31 carry each row's total into the rows above.
__device__ __forceinline__ int wave_scan_add_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}

struct f3x2 {
    v2 x, y, z;
};

__device__ __forceinline__ v2 vfma(v2 a, v2 b, v2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2 vmax(v2 a, v2 b) { return __builtin_elementwise_max(a, b); }  // IEEE maxNum
__device__ __forceinline__ v2 vmin(v2 a, v2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ v2 vsat(v2 a) { return vmin(vmax(a, (v2)(0.0f)), (v2)(1.0f)); }
__device__ __forceinline__ v2 vsel(m2 m, v2 a, v2 b) { return v2{on(m.x) ? a.x : b.x, on(m.y) ? a.y : b.y}; }
__device__ __forceinline__ m2 ge(v2 a, float c) { return mask2(a.x >= c, a.y >= c); }
__device__ __forceinline__ m2 le(v2 a, float c) { return mask2(a.x <= c, a.y <= c); }
__device__ __forceinline__ m2 eq(v2 a, float c) { return mask2(a.x == c, a.y == c); }
__device__ __forceinline__ m2 not_gt(v2 a, float c) { return mask2(!(a.x > c), !(a.y > c)); }
__device__ __forceinline__ f3x2 add3(f3x2 a, f3x2 b) { return f3x2{a.x + b.x, a.y + b.y, a.z + b.z}; }
// HLSL dot, same association as dot3: (a.x*b.x + a.y*b.y) + a.z*b.z
__device__ __forceinline__ v2 dot3(f3x2 a, f3x2 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v2 splat(float s) { return (v2)(s); }
__device__ __forceinline__ f3x2 splat3(float x, float y, float z) { return f3x2{splat(x), splat(y), splat(z)}; }
__device__ __forceinline__ f3 lane(const f3x2& v, int i) { return i ? mk3(v.x.y, v.y.y, v.z.y) : mk3(v.x.x, v.y.x, v.z.x); }

// saturate(dot(a, b)) with the saturate folded into the dot's last packed add as its clamp bit
// (v_pk_add_f32 ... clamp: the IEEE sum, then clamped to [0, 1]; DX10_CLAMP maps NaN to 0, as HLSL's
// saturate does). The compiler applies the clamp as a separate v_max per element. Inline asm: the
// s_nop 1 pads keep two wait states on both sides, whatever hazard the neighbours would need.
__device__ __forceinline__ v2 dot3_sat(f3x2 a, f3x2 b) {
    const v2 t = a.x * b.x + a.y * b.y, u = a.z * b.z;
    v2 r;
    asm("s_nop 1\n\tv_pk_add_f32 %0, %1, %2 clamp\n\ts_nop 1" : "=v"(r) : "v"(t), "v"(u));
    return r;
}

struct Recip2 {
    v2 y, r;
};
__device__ __forceinline__ Recip2 recip_nr(v2 y) {
    v2 r = v2{__builtin_amdgcn_rcpf(y.x), __builtin_amdgcn_rcpf(y.y)};
    v2 e = vfma(-y, r, splat(1.0f));
    return Recip2{y, vfma(e, r, r)};
}
__device__ __forceinline__ v2 div_nr(v2 x, Recip2 d) {  // Markstein step, see pbr_device_math.h
    v2 q = x * d.r;
    v2 t = vfma(d.y, q, -x);
    return vfma(-t, d.r, q);
}
__device__ __forceinline__ v2 sqrt_nr(v2 x) {  // see sqrt_nr in pbr_device_math.h
    const v2 y = v2{__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)};
    const v2 s0 = x * y;
    const v2 r = vfma(-s0, s0, x);
    return vfma(r, 0.5f * y, s0);
}
// pow5_light for the pair, element for element the same values: the fp64 products of both elements unconditionally
// (straight-line: the compiler interleaves the two chains with the work around them, where a per-element branch kept
// each chain in its own block), glibc's algorithm patched in above PBR_POW5_GLIBC_FROM under a wave-uniform branch
// taken only when a lane of `live` (the lanes whose result is used) needs it.
__device__ __forceinline__ v2 pow5_light(v2 x, uint64_t live = ~0ull) {
    const double dx = (double)x.x, dy = (double)x.y;
    const double dx2 = dx * dx, dy2 = dy * dy;
    v2 p = v2{(float)(dx2 * dx2 * dx), (float)(dy2 * dy2 * dy)};
    // Two ballots of the compares themselves: a ballot of their || was formed through a VGPR (v_cndmask, v_cmp_ne).
    if (__builtin_expect(((lanes(x.x > PBR_POW5_GLIBC_FROM) | lanes(x.y > PBR_POW5_GLIBC_FROM)) & live) != 0, 0)) {
        if (x.x > PBR_POW5_GLIBC_FROM && on(live)) p.x = pow5_glibc(x.x);
        if (x.y > PBR_POW5_GLIBC_FROM && on(live)) p.y = pow5_glibc(x.y);
    }
    return p;
}
// |x| in [lo, hi] per element (false for NaN).
__device__ __forceinline__ m2 in_win(v2 x, float lo, float hi) {
    v2 a = __builtin_elementwise_abs(x);
    return ge(a, lo) & le(a, hi);
}

struct PixelInvariants2 {
    f3x2 n, v, albedo, f0, one_minus_f0;
    v2 one_minus_metal, a_sqr, a_sqr_minus_1, k, one_minus_k, ggx_v, four_n_dot_v;
    m2 f0_nonzero;  // no F0 component is zero
};

// make_invariants (pbr_device_math.h) element-wise for the pair: the same operations, packed. The one
// division, GeometrySchlickGGX(N.V) = n_dot_v / (n_dot_v (1-k) + k), takes the Markstein step for
// pixels in the fast window (`fast`): roughness in [0, 1] puts k in [1/8, 1/2] and the denominator in
// [2^-3, 2^5]; n_dot_v must be 0 or >= 2^-100 so the residual stays normal. Otherwise IEEE.
__device__ __forceinline__ PixelInvariants2 complete_invariants(PixelInvariants2 q, v2 roughness, m2 fast);
__device__ __forceinline__ PixelInvariants2 make_invariants(const f3x2& n, const f3x2& v, const f3x2& albedo,
                                                            const f3x2& f0, v2 metallic, v2 roughness, m2 fast) {
    PixelInvariants2 q;
    q.n = n;
    q.v = v;
    q.albedo = albedo;
    q.f0 = f0;
    q.one_minus_f0 = f3x2{1.0f - f0.x, 1.0f - f0.y, 1.0f - f0.z};
    q.one_minus_metal = 1.0f - metallic;
    return complete_invariants(q, roughness, fast);
}
// make_invariants' light-loop fields (a^2, k, GeometrySchlickGGX(N.V), 4 N.V) from q's N and V and the roughness.
__device__ __forceinline__ PixelInvariants2 complete_invariants(PixelInvariants2 q, v2 roughness, m2 fast) {
    const f3x2 n = q.n, v = q.v, f0 = q.f0;
    v2 r = vmax(roughness, splat(0.05f));
    v2 a = r * r;
    q.a_sqr = a * a;
    q.a_sqr_minus_1 = q.a_sqr - 1.0f;
    v2 rr = (roughness + 1.0f);
    q.k = (rr * rr) * 0.125f;  // (r*r) / 8.0f: division by a power of two is this exact product
    q.one_minus_k = 1.0f - q.k;
    v2 n_dot_v = vmax(dot3(n, v), splat(0.0f));
    const v2 den = n_dot_v * q.one_minus_k + q.k;
    const m2 ok = fast & (eq(n_dot_v, 0.0f) | ge(n_dot_v, 0x1p-100f));
    const v2 gq = div_nr(n_dot_v, recip_nr(den));
    if (__builtin_expect(on(ok.x) && on(ok.y), 1)) {
        q.ggx_v = gq;
    } else {
        q.ggx_v = v2{on(ok.x) ? gq.x : n_dot_v.x / den.x, on(ok.y) ? gq.y : n_dot_v.y / den.y};
    }
    q.four_n_dot_v = 4.0f * n_dot_v;
    q.f0_nonzero = mask2(f0.x.x != 0.0f && f0.y.x != 0.0f && f0.z.x != 0.0f,
                         f0.x.y != 0.0f && f0.y.y != 0.0f && f0.z.y != 0.0f);
    return q;
}

// The fields of make_invariants the finish reads (Default.hlsl:139-150: the ambient's N, V, F0, 1 - F0, 1 - metallic,
// albedo), by the same operations, so the same bits; the light-loop fields (a^2, k, GeometrySchlickGGX(N.V), 4 N.V)
// are left zero. The wave-balanced kernels form these after their loop; the rare exact re-pass forms the full set.
__device__ __forceinline__ PixelInvariants2 make_finish_invariants(const f3x2& n, const f3x2& v, const f3x2& albedo,
                                                                   const f3x2& f0, v2 metallic) {
    PixelInvariants2 q{};
    q.n = n;
    q.v = v;
    q.albedo = albedo;
    q.f0 = f0;
    q.one_minus_f0 = f3x2{1.0f - f0.x, 1.0f - f0.y, 1.0f - f0.z};
    q.one_minus_metal = 1.0f - metallic;
    return q;
}

// normalize3 (IEEE sqrtf and division) on each element of the pair.
__device__ __forceinline__ f3x2 normalize_ieee(const f3x2& v) {
    const f3 a = normalize3(lane(v, 0)), b = normalize3(lane(v, 1));
    return f3x2{v2{a.x, b.x}, v2{a.y, b.y}, v2{a.z, b.z}};
}

// Scalar PixelInvariants of pixel i of the pair (for the exact fallback).
__device__ __forceinline__ PixelInvariants unpack_invariants(const PixelInvariants2& q, int i) {
    PixelInvariants s;
    s.n = lane(q.n, i);
    s.v = lane(q.v, i);
    s.albedo = lane(q.albedo, i);
    s.f0 = lane(q.f0, i);
    s.one_minus_f0 = lane(q.one_minus_f0, i);
    s.one_minus_metal = i ? q.one_minus_metal.y : q.one_minus_metal.x;
    s.a_sqr = i ? q.a_sqr.y : q.a_sqr.x;
    s.a_sqr_minus_1 = i ? q.a_sqr_minus_1.y : q.a_sqr_minus_1.x;
    s.k = i ? q.k.y : q.k.x;
    s.one_minus_k = i ? q.one_minus_k.y : q.one_minus_k.x;
    s.ggx_v = i ? q.ggx_v.y : q.ggx_v.x;
    s.four_n_dot_v = i ? q.four_n_dot_v.y : q.four_n_dot_v.x;
    s.fast_ok = false;
    s.f0_nonzero = on(i ? q.f0_nonzero.y : q.f0_nonzero.x);
    return s;
}

// BRDFCookTorrance, packed fast path (scalar twin: brdf_cook_torrance<true>). `ok` collects the
// per-iteration window conditions (see pbr_device_math.h).
__device__ __forceinline__ v2 div_pi(v2 x) { return vfma(x, splat(kInvPiHi), x * kInvPiLo); }  // see div_pi

// LEAN: every pixel of the wave is inside the fast window with |N|^2 <= 1 + 2^-20 (dot3 as rounded)
// and no zero F0 component; then two of the per-light window tests hold without being tested:
//  * den: |N| <= 1 + 2^-20.9 and the fast normalize gives |H| <= 1 + 2^-21, so N.H <= 1 + 2^-19.6
//    after the dot's roundings and n_dot_h^2 <= 1 + 2^-18.6; with roughness clamped to >= 0.05,
//    a^2 >= 2^-17.29 and inner = n_dot_h^2 (a^2 - 1) + 1 >= a^2 - 2^-18.6 (1 - a^2) - 2^-23 >= 2^-18.1,
//    inner <= 1, so den = pi inner^2 is in [2^-37, pi], inside [2^-60, 2^60];
//  * with |F0| in [2^-20, 1024] (per-pixel window, no zero component), F = F0 + (1 - F0) p is either
//    near F0 or an exact cancellation (a multiple of ulp(F0)/2 >= 2^-45), so F is 0 or >= 2^-45 and
//    ndf_g F stays inside the division window for any p: the p == 0 / p >= 2^-40 test is moot.
//
// QUARTER (lean only; the exact wave-balanced items, pbr_balanced.h): q carries N / 4, k / 4 (1 - k as it is),
// 16 (a^2 - 1), 16 N.V in place of 4 N.V, and `radiance` is 4x the reference's -- all exact power-of-two scalings, so
// max(N.H, 0) / 4 and max(N.L, 0) / 4 come out of the dots bit for bit (every product of them is 0 or >= 2^-110 in
// the window) and below 1 in lean waves, where they ride on the dot's clamp bit instead of a v_max per element; the
// quarters cancel against the scaled invariants in every later operation (N.H^2 / 16 x 16 (a^2 - 1); N.L / 4 over
// N.L (1 - k) / 4 + k / 4; 16 N.V x N.L / 4; 4 radiance x N.L / 4), so each value is the unscaled loop's bit for bit.
template <bool LEAN, bool QUARTER = false>
__device__ __forceinline__ f3x2 brdf_x2(const PixelInvariants2& q, f3x2 radiance, f3x2 l, f3x2 h, m2& ok,
                                        uint64_t live = ~0ull) {
    static_assert(LEAN || !QUARTER, "the clamp form needs the lean bounds |N|, |H|, |L| <= 1 + 2^-19");
    v2 n_dot_h = QUARTER ? dot3_sat(q.n, h) : vmax(dot3(q.n, h), splat(0.0f));
    v2 n_dot_h_sqr = n_dot_h * n_dot_h;
    v2 den = (n_dot_h_sqr * q.a_sqr_minus_1 + 1.0f);
    den = kPi * den * den;
    if (!LEAN) ok &= ge(den, 0x1p-60f) & le(den, 0x1p60f);
    v2 ndf = div_nr(q.a_sqr, recip_nr(den));
    v2 n_dot_l = QUARTER ? dot3_sat(q.n, l) : vmax(dot3(q.n, l), splat(0.0f));
    v2 ggx_l = div_nr(n_dot_l, recip_nr(n_dot_l * q.one_minus_k + q.k));
    v2 g = ggx_l * q.ggx_v;
    v2 cos_theta = dot3_sat(h, q.v);
    v2 p = pow5_light(1.0f - cos_theta, live);
    f3x2 f = f3x2{q.f0.x + q.one_minus_f0.x * p, q.f0.y + q.one_minus_f0.y * p, q.f0.z + q.one_minus_f0.z * p};
    v2 ndf_g = ndf * g;
    v2 denom = q.four_n_dot_v * n_dot_l + 0.001f;
    f3x2 nom = f3x2{ndf_g * f.x, ndf_g * f.y, ndf_g * f.z};
    if (LEAN) {
        // ndf_g is +-0 or positive here (a^2 > 0, den > 0, N.L and ggx_v >= 0) and at most 2^38
        // (ndf <= a^2 / 2^-37 <= 2^37; ggx_l, ggx_v <= 1 + 2^-19 for |N.L|, |N.V| <= 1 + 2^-19), so the
        // window is "0 or >= 2^-30": one integer op and one compare on the bit pattern, b - 1 >= bits(2^-30) - 1
        // (unsigned; +0 wraps to the maximum, -0 is 0x80000000 and passes too).
        // Element bits through __float_as_uint (a by-value copy): this clang reads element 0 for
        // __builtin_bit_cast(uint32_t, v.y) on an ext_vector_type element (compiler notes).
        const uint32_t bx = __float_as_uint(ndf_g.x) - 1u, by = __float_as_uint(ndf_g.y) - 1u;
        ok &= mask2(bx >= 0x30800000u - 1u, by >= 0x30800000u - 1u);
    } else {
        ok &= eq(ndf_g, 0.0f) | in_win(ndf_g, 0x1p-30f, 0x1p40f);
        ok &= q.f0_nonzero | eq(p, 0.0f) | ge(p, 0x1p-40f);
    }
    const Recip2 rd = recip_nr(denom);
    f3x2 spec = f3x2{div_nr(nom.x, rd), div_nr(nom.y, rd), div_nr(nom.z, rd)};
    f3x2 kd = f3x2{(1.0f - f.x) * q.one_minus_metal, (1.0f - f.y) * q.one_minus_metal, (1.0f - f.z) * q.one_minus_metal};
    return f3x2{((div_pi(kd.x * q.albedo.x) + spec.x) * radiance.x) * n_dot_l,
                ((div_pi(kd.y * q.albedo.y) + spec.y) * radiance.y) * n_dot_l,
                ((div_pi(kd.z * q.albedo.z) + spec.z) * radiance.z) * n_dot_l};
}

__device__ __forceinline__ f3x2 normalize_x2(f3x2 v, m2& ok) {
    v2 s = sqrt_nr(dot3(v, v));
    ok &= ge(s, 0x1p-30f);  // s <= 1 + |L| <= 29 by the windows
    const Recip2 r = recip_nr(s);
    return f3x2{div_nr(v.x, r), div_nr(v.y, r), div_nr(v.z, r)};
}

// ComputeDirectionalLight, packed fast path.
template <bool LEAN>
__device__ __forceinline__ f3x2 directional_x2(const PixelInvariants2& q, float4 s, float4 d, m2& ok) {
    f3x2 l = splat3(-d.x, -d.y, -d.z);
    f3x2 h = normalize_x2(add3(q.v, l), ok);
    return brdf_x2<LEAN>(q, splat3(s.x, s.y, s.z), l, h, ok);
}

// max(x, 0.01f) of CalcAttenuation (LightingUtil.hlsl:38) as one v_med3_f32(x, 0.01, 2^100): the
// same value as maxNum for every x <= 2^100 (an in-window distance is below 2^22), without the
// quieting v_max the compiler puts in front of an IEEE-mode v_max_f32 whose input it cannot prove
// canonical (with +inf as the bound the intrinsic is folded back into that maxnum). A NaN or huge
// distance fails the window (ge(dist, 2^-20) / the position windows), so that lane is redone on the
// exact path whatever this returns.
__device__ __forceinline__ v2 max_dsat(v2 dist) {
    return v2{__builtin_amdgcn_fmed3f(dist.x, 0.01f, 0x1p100f),
              __builtin_amdgcn_fmed3f(dist.y, 0.01f, 0x1p100f)};
}

// The range test of ComputePointLight (LightingUtil.hlsl:131: d > 100 adds nothing) as a factor of exactly
// 1 or 0: floats next to 100 are 2^-17 apart, so d <= 100 <=> 2^17 (100 + 2^-17 - d) >= 1 and d > 100 <=> it
// is <= 0. One v_pk_fma forms that product with a single rounding (-2^17 d is exact, 2^17 (100 + 2^-17) =
// 13107201 is a float) and its clamp bit maps it to 1 or 0 (NaN to 0: such a lane fails the window). Both
// constants come from one SGPR pair (op_sel picks the half: one constant-bus read). Replaces the two
// compares and two selects of a lit mask. s_nop pads as in dot3_sat.
__device__ __forceinline__ v2 in_range01(v2 dist) {
    const v2 kc = v2{-0x1p17f, 13107201.0f};
    v2 r;
    asm("s_nop 1\n\tv_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1] clamp\n\ts_nop 1"
        : "=v"(r) : "v"(dist), "s"(kc));
    return r;
}

// The range test for spot lights: a select, not the 0/1 factor. The cone factor pow(c, SpotPower)
// (LightingUtil.hlsl:163) can be +inf or NaN for an adversarial light (SpotPower < 0 with c = 0, a NaN
// SpotPower, |Direction| > 1 under a huge power) that the light window does not see, and inf * 0 = NaN,
// where the reference returns 0 before it evaluates the pow (:154). Spot lights already pay two glibc
// powf per pair, so the select costs nothing measurable.
__device__ __forceinline__ v2 spot_range_select(v2 att, v2 dist) {
    return v2{dist.x > 100.0f ? 0.0f : att.x, dist.y > 100.0f ? 0.0f : att.y};
}

// ComputePointLight / ComputeSpotLight, packed fast path. The range test (exact, as in the scalar
// version) scales the attenuation by 1 or 0 (in_range01), so an unlit lane's contribution is
// (finite) * 0 = +-0 whenever the lane is inside the window (`ok`: every value of the fast path is then
// finite; pbr_set_pass clears the light's window flag when its strength is not finite), and adding +-0
// to the running sum is the identity the reference's skipped light is. Lanes outside the window are
// redone by the caller whether lit or not.
template <bool SPOT, bool LEAN>
__device__ __forceinline__ f3x2 point_or_spot_x2(const PixelInvariants2& q, const f3x2& pos,
                                                 float4 s, float4 d, float4 p, m2& ok) {
    f3x2 l = f3x2{p.x - pos.x, p.y - pos.y, p.z - pos.z};
    v2 dist = sqrt_nr(dot3(l, l));
    ok &= ge(dist, 0x1p-20f);
    const Recip2 rdist = recip_nr(dist);
    l = f3x2{div_nr(l.x, rdist), div_nr(l.y, rdist), div_nr(l.z, rdist)};
    f3x2 h = normalize_x2(add3(q.v, l), ok);
    v2 dsat = max_dsat(dist);
    v2 att = recip_nr(dsat * dsat).r;  // RN(1/y) already (see point_or_spot_light)
    if (SPOT) {
        v2 c = vmax(dot3(f3x2{-l.x, -l.y, -l.z}, splat3(d.x, d.y, d.z)), splat(0.0f));
        att *= v2{powf_glibc(c.x, s.w), powf_glibc(c.y, s.w)};
        att = spot_range_select(att, dist);
    } else {
        att *= in_range01(dist);  // beyond the range: +0
    }
    return brdf_x2<LEAN>(q, f3x2{s.x * att, s.y * att, s.z * att}, l, h, ok);
}

// ---- PBR_FLAG_FAITHFUL: the tolerance-mode light loop (lean waves only) --------------------------------
//
// Exact, as in the default mode: everything upstream of the two ill-conditioned spots -- L, dist,
// H = normalize(V + L), N.H and the GGX denominator `den` -- and the Fresnel term F, whose 1 - F cancels
// at grazing angles. Rearranged, with the error bounded instead of bit-matched: the well-conditioned
// rest of BRDFCookTorrance and the attenuation,
//
//   spec.c = NDF * G * F.c / denom = F.c * (a^2 * G1(N.V) * N.L / PI) / (inner^2 * (N.L (1-k) + k) * denom)
//   diff.c = (1 - F.c) * (1 - metallic) * albedo.c / PI
//   sum.c += (diff.c + spec.c) * strength.c * (att * N.L),     att = min(RN(1/dist)^2, 1/0.01^2)
//
// (inner = N.H^2 (a^2 - 1) + 1, the GGX denominator before its PI and square) with one hardware
// reciprocal (<= 1 ulp) for the three denominators, the per-pixel products a^2 * G1(N.V) / PI and
// (1 - metallic) * albedo / PI hoisted out of the loop, and fused multiply-adds (single roundings) for the
// Smith and specular denominators, the diffuse term, the diffuse + specular sum and the accumulation.
// Untiled passes run the loop on invariants rescaled by powers of two (faithful_scale): N / 4, so that
// max(N.H, 0) and max(N.L, 0) come out / 4 and, in lean waves, ride on the dot's clamp bit instead of a
// v_max per element -- exactly, because the fast window keeps every product of those dots 0 or >= 2^-110 --
// with the 4s folded back into the other per-pixel factors; each light's term then stays within 26
// roundings (2^-24 each) of the reference's. Tiled passes keep the first form (PI * inner^2, the reference's
// roundings of the two denominators, N.L saturated in lean waves): within 38 roundings. With every term >= 0
// (host: strengths, ambient, env texels >= 0, <= 64 summed terms; per wave: albedo >= 0, F0 in [0, 1]) the
// output is within 5.5e-6 (untiled) / 5.9e-6 (tiled) relative with the faithful finish --
// inside the north-star 1e-5 -- but not bit-identical.
__device__ __forceinline__ v2 rcp_hw(v2 y) { return v2{__builtin_amdgcn_rcpf(y.x), __builtin_amdgcn_rcpf(y.y)}; }
constexpr float kInvPi = 0x1.45f306p-2f;  // RN(1/kPi)

// Fresnel x^5 of the faithful loop: compensated fp32 arithmetic in packed form (x^2 and x2^2 split exactly
// by FMA, the cross term 2 x2 e2 folded in, one final rounding) -- within 2^-45 of x^5 before rounding,
// so within 0.5 ulp + 2^-22 ulp of it and at most 1 ulp from glibc's powf (0.82 ulp), the same residue
// the exact mode's fp64 x^5 has (pow5_light; DESIGN.md §2 counts it). 8 packed ops per pair instead of
// 10 fp64 ones. The grazing band x > 0.99, where 1 - F cancels, keeps glibc's algorithm bit for bit.
// `live`: the lanes whose result is used (the wave-balanced loop runs every lane, finished ones on zero-strength
// sentinel items); the grazing branch is taken only for them.
__device__ __forceinline__ v2 pow5_faithful(v2 x, uint64_t live = ~0ull) {
    const v2 x2 = x * x;
    const v2 e2 = vfma(x, x, -x2);
    const v2 x4 = x2 * x2;
    const v2 t = vfma(x2 + x2, e2, vfma(x2, x2, -x4));
    v2 p = vfma(x4, x, t * x);
    if (__builtin_expect((lanes(x.x > PBR_POW5_GLIBC_FROM) & live) != 0, 0)) {
        if (x.x > PBR_POW5_GLIBC_FROM && on(live)) p.x = pow5_glibc(x.x);
    }
    if (__builtin_expect((lanes(x.y > PBR_POW5_GLIBC_FROM) & live) != 0, 0)) {
        if (x.y > PBR_POW5_GLIBC_FROM && on(live)) p.y = pow5_glibc(x.y);
    }
    return p;
}

// Fresnel x^5 of the wave-balanced faithful items (pbr_balanced.h, pass 2): three plain products, x^2, x^4, x^5
// (each rounded once: within 4u + 6u^2 of x^5, u = 2^-24, so within 5.64u p of glibc's powf, which is within 0.82 ulp
// <= 1.64u p of x^5), 3 packed ops per pair instead of pow5_faithful's 8. The diffuse factor 1 - F = (1 - F0)(1 - p)
// sees that difference amplified by p / (1 - p), so glibc's algorithm takes over above x = 0.97 (p = 0.859, factor
// 6.1): <= 5.64u * 6.1 = 34.4u = 2.05e-6 on a term's diffuse part (pow5_faithful: 1 ulp, <= 1.2e-6 below 0.99; the
// bound of DESIGN.md §2 carries the difference). Above 0.97, H.V < 0.03: L within ~3.4 degrees of -V, which a live
// item (N.L > 0, N.V >= 0) reaches only at grazing views, so the branch stays rare. `live` as in pow5_faithful.
#ifndef PBR_POW5_FAST3_GLIBC_FROM
#define PBR_POW5_FAST3_GLIBC_FROM 0.97f
#endif
__device__ __forceinline__ v2 pow5_fast3(v2 x, uint64_t live) {
    const v2 x2 = x * x;
    const v2 x4 = x2 * x2;
    v2 p = x4 * x;
    if (__builtin_expect((lanes(x.x > PBR_POW5_FAST3_GLIBC_FROM) & live) != 0, 0)) {
        if (x.x > PBR_POW5_FAST3_GLIBC_FROM && on(live)) p.x = pow5_glibc(x.x);
    }
    if (__builtin_expect((lanes(x.y > PBR_POW5_FAST3_GLIBC_FROM) & live) != 0, 0)) {
        if (x.y > PBR_POW5_FAST3_GLIBC_FROM && on(live)) p.y = pow5_glibc(x.y);
    }
    return p;
}

// SCALED (the untiled kernels): the loop runs on invariants rescaled by powers of two (faithful_scale) and
// the Smith and specular denominators are FMAs. Unscaled (tiled culling, where a wave sums a handful of
// lights and the per-pixel rescaling does not pay for itself; measured 4% slower on config 4) keeps the
// first form: N.L saturated in lean waves, PI * inner^2, the two denominators as the reference rounds them.
struct Faithful2 {
    v2 a2gv;     // a^2 * GeometrySchlickGGX(N.V), SCALED: * 16 / PI (4 for N.L / 4, 4 for the scaled sum)
    f3x2 mabpi;  // (1 - metallic) * albedo / PI, SCALED: * 4
};
constexpr float kInvPi4 = 4.0f * kInvPi, kInvPi16 = 16.0f * kInvPi;  // exact scalings of RN(1/kPi)
template <bool SCALED>
__device__ __forceinline__ Faithful2 make_faithful(const PixelInvariants2& q) {
    const float c = SCALED ? kInvPi4 : kInvPi;
    return Faithful2{SCALED ? (q.a_sqr * q.ggx_v) * kInvPi16 : q.a_sqr * q.ggx_v,
                     f3x2{(q.one_minus_metal * q.albedo.x) * c, (q.one_minus_metal * q.albedo.y) * c,
                          (q.one_minus_metal * q.albedo.z) * c}};
}

// The SCALED loop's invariants: N / 4, 16 (a^2 - 1), 4 (1 - k), 16 N.V. Every factor is a power of two and
// every value is 0 or normal far from both ends in the fast window (normal components 0 or in [2^-20, 16],
// a^2 - 1 in [-1, 0] with |a^2 - 1| 0 or >= 2^-24, 1 - k in [1/2, 7/8], N.V 0 or >= 2^-100), so scaling is
// exact and faithful_unscale restores the bits the exact re-pass and the finish read. With V + L components
// 0 or >= 2^-88 (and L/d >= 2^-65) the products of N/4 . H and N/4 . L stay 0 or >= 2^-110: no subnormal
// rounding anywhere in those dots, so each is exactly a quarter of the reference's dot.
__device__ __forceinline__ void faithful_scale(PixelInvariants2& q) {
    q.n = f3x2{q.n.x * 0.25f, q.n.y * 0.25f, q.n.z * 0.25f};
    q.a_sqr_minus_1 *= 16.0f;
    q.one_minus_k *= 4.0f;
    q.four_n_dot_v *= 4.0f;
}
__device__ __forceinline__ void faithful_unscale(PixelInvariants2& q) {
    q.n = f3x2{q.n.x * 4.0f, q.n.y * 4.0f, q.n.z * 4.0f};
    q.a_sqr_minus_1 *= 0.0625f;
    q.one_minus_k *= 0.25f;
    q.four_n_dot_v *= 0.25f;
}

// BRDFCookTorrance * radiance * N.L added into `sum`; `att` = the light's attenuation (1 for directional
// lights), already 0 for lanes beyond the range. LEAN as in brdf_x2: outside lean waves (|N| up to the
// window's bound, zero F0 components) N.H and N.L take max(., 0) (no clamp bit: their quarter may exceed
// 1), and the GGX denominator is tested so that the product of the three denominators stays normal.
template <bool LEAN, bool SCALED>
__device__ __forceinline__ void brdf_faithful_x2(const PixelInvariants2& q, const Faithful2& fi, float4 s, v2 att,
                                                 f3x2 l, f3x2 h, m2& ok, f3x2& sum) {
    // SCALED: max(N.H, 0) / 4 and max(N.L, 0) / 4, bit for bit. Lean waves: |N|, |H|, |L| <= 1 + 2^-19.6, so
    // the quarter is below 1 and the [0, 1] clamp of the dot's last add is max(., 0). Unscaled lean waves
    // saturate N.L instead of max(., 0): N.L is not on the ill-conditioned chain, and there it exceeds 1 by
    // at most 2^-20.6, a relative change the bound absorbs.
    const v2 n_dot_h = (SCALED && LEAN) ? dot3_sat(q.n, h) : vmax(dot3(q.n, h), splat(0.0f));
    const v2 inner = ((n_dot_h * n_dot_h) * q.a_sqr_minus_1 + 1.0f);  // exact: the ill-conditioned GGX denominator
    const v2 den = SCALED ? inner * inner : kPi * inner * inner;      // SCALED: the NDF's denominator / PI
    if (!LEAN) ok &= SCALED ? ge(den, 0x1p-62f) & le(den, 0x1p58f) : ge(den, 0x1p-60f) & le(den, 0x1p60f);
    const v2 n_dot_l = LEAN ? dot3_sat(q.n, l) : vmax(dot3(q.n, l), splat(0.0f));
    const v2 r = SCALED ? rcp_hw((den * vfma(n_dot_l, q.one_minus_k, q.k)) * vfma(q.four_n_dot_v, n_dot_l, splat(0.001f)))
                        : rcp_hw((den * (n_dot_l * q.one_minus_k + q.k)) * (q.four_n_dot_v * n_dot_l + 0.001f));
    const v2 p = pow5_faithful(1.0f - dot3_sat(h, q.v));
    const f3x2 f = f3x2{q.f0.x + q.one_minus_f0.x * p, q.f0.y + q.one_minus_f0.y * p, q.f0.z + q.one_minus_f0.z * p};
    const v2 kr = (fi.a2gv * n_dot_l) * r;  // SCALED: 4 x the specular factor
    const v2 w = att * n_dot_l;             // SCALED: att * N.L / 4
    sum.x = vfma(vfma(kr, f.x, vfma(-f.x, fi.mabpi.x, fi.mabpi.x)), s.x * w, sum.x);
    sum.y = vfma(vfma(kr, f.y, vfma(-f.y, fi.mabpi.y, fi.mabpi.y)), s.y * w, sum.y);
    sum.z = vfma(vfma(kr, f.z, vfma(-f.z, fi.mabpi.z, fi.mabpi.z)), s.z * w, sum.z);
}

template <bool LEAN, bool SCALED>
__device__ __forceinline__ void directional_faithful_x2(const PixelInvariants2& q, const Faithful2& fi, float4 s,
                                                        float4 d, m2& ok, f3x2& sum) {
    const f3x2 l = splat3(-d.x, -d.y, -d.z);
    const f3x2 h = normalize_x2(add3(q.v, l), ok);
    brdf_faithful_x2<LEAN, SCALED>(q, fi, s, splat(1.0f), l, h, ok, sum);
}

template <bool SPOT, bool LEAN, bool SCALED>
__device__ __forceinline__ void point_or_spot_faithful_x2(const PixelInvariants2& q, const Faithful2& fi,
                                                          const f3x2& pos, float4 s, float4 d, float4 p, m2& ok,
                                                          f3x2& sum) {
    f3x2 l = f3x2{p.x - pos.x, p.y - pos.y, p.z - pos.z};
    const v2 dist = sqrt_nr(dot3(l, l));
    // Window: dist >= 0.01 (stricter than the exact loop's 2^-20). Then max(dist, 0.01) of CalcAttenuation
    // (LightingUtil.hlsl:35-40) is dist itself and the attenuation is RN(1/dist)^2 from the correctly rounded
    // reciprocal the exact L already needs; a pixel closer than 0.01 to a light is redone exactly.
    ok &= ge(dist, 0.01f);
    const Recip2 rdist = recip_nr(dist);
    l = f3x2{div_nr(l.x, rdist), div_nr(l.y, rdist), div_nr(l.z, rdist)};
    const f3x2 h = normalize_x2(add3(q.v, l), ok);
    v2 att = rdist.r * rdist.r;
    if (SPOT) {
        const v2 c = vmax(dot3(f3x2{-l.x, -l.y, -l.z}, splat3(d.x, d.y, d.z)), splat(0.0f));
        att *= v2{powf_glibc(c.x, s.w), powf_glibc(c.y, s.w)};
        att = spot_range_select(att, dist);
    } else {
        att *= in_range01(dist);  // beyond the range: +0 (see point_or_spot_x2)
    }
    brdf_faithful_x2<LEAN, SCALED>(q, fi, s, att, l, h, ok, sum);
}

}  // namespace pbr
