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

constexpr float kPi = 3.14159265359f;  // LightingUtil.hlsl:59, 103 (an fp32 literal in HLSL)
constexpr float kInvGamma = 1.0f / 2.2f;  // Default.hlsl:155
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
};

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
    return q;
}

// BRDFCookTorrance (LightingUtil.hlsl:85-104) with DistributionGGX (:49-62), GeometrySmith (:75-83)
// and FresnelSchlick (:43-47) inlined; returns (kD*albedo/PI + specular) * radiance * NdotL.
__device__ __forceinline__ f3 brdf_cook_torrance(const PixelInvariants& q, f3 radiance, f3 l, f3 h) {
    // DistributionGGX
    float n_dot_h = hmax(dot3(q.n, h), 0.0f);
    float n_dot_h_sqr = n_dot_h * n_dot_h;
    float den = (n_dot_h_sqr * q.a_sqr_minus_1 + 1.0f);
    den = kPi * den * den;
    float ndf = q.a_sqr / den;
    // GeometrySmith: ggx1 * ggx2
    float n_dot_l = hmax(dot3(q.n, l), 0.0f);
    float ggx_l = n_dot_l / (n_dot_l * q.one_minus_k + q.k);
    float g = ggx_l * q.ggx_v;
    // FresnelSchlick(H, V, F0)
    float cos_theta = hsat(dot3(h, q.v));
    float p = powf(1.0f - cos_theta, 5.0f);
    f3 f = mk3(q.f0.x + q.one_minus_f0.x * p, q.f0.y + q.one_minus_f0.y * p, q.f0.z + q.one_minus_f0.z * p);
    // specular = (NDF*G)*F / (4*NdotV*NdotL + 0.001)
    float ndf_g = ndf * g;
    float denom = q.four_n_dot_v * n_dot_l + 0.001f;
    f3 spec = mk3((ndf_g * f.x) / denom, (ndf_g * f.y) / denom, (ndf_g * f.z) / denom);
    // kD = (1 - F) * (1 - metallic)
    f3 kd = mk3((1.0f - f.x) * q.one_minus_metal, (1.0f - f.y) * q.one_minus_metal, (1.0f - f.z) * q.one_minus_metal);
    return mk3((((kd.x * q.albedo.x) / kPi + spec.x) * radiance.x) * n_dot_l,
               (((kd.y * q.albedo.y) / kPi + spec.y) * radiance.y) * n_dot_l,
               (((kd.z * q.albedo.z) / kPi + spec.z) * radiance.z) * n_dot_l);
}

// ComputeDirectionalLight (LightingUtil.hlsl:109-119). The caller adds shadowFactor(1,1,1) * result,
// and 1.0f * x == x exactly, so the multiply is omitted.
__device__ __forceinline__ f3 directional_light(const PixelInvariants& q, float4 s, float4 d) {
    f3 l = mk3(-d.x, -d.y, -d.z);
    f3 h = normalize3(add3(q.v, l));
    return brdf_cook_torrance(q, mk3(s.x, s.y, s.z), l, h);
}

// ComputePointLight (:124-142) / ComputeSpotLight (:147-167). Returns false when the range test at
// :131 / :154 returns 0: adding +0 to the running sum is the identity (the sum starts at +0 and is
// never -0), so skipping it is bit-exact.
template <bool SPOT>
__device__ __forceinline__ bool point_or_spot_light(const PixelInvariants& q, f3 pos, float4 s, float4 d, float4 p,
                                                    f3& out) {
    f3 l = mk3(p.x - pos.x, p.y - pos.y, p.z - pos.z);
    float dist = sqrtf(dot3(l, l));
    if (dist > kLightRange) return false;
    l = mk3(l.x / dist, l.y / dist, l.z / dist);
    f3 h = normalize3(add3(q.v, l));
    float dsat = hmax(dist, 0.01f);  // CalcAttenuation (:35-40)
    float att = 1.0f / (dsat * dsat);
    if (SPOT) {
        f3 nl = mk3(-l.x, -l.y, -l.z);
        att *= powf(hmax(dot3(nl, mk3(d.x, d.y, d.z)), 0.0f), s.w);  // :163, SpotPower in .w
    }
    out = brdf_cook_torrance(q, mk3(s.x * att, s.y * att, s.z * att), l, h);
    return true;
}

// WorldToSkyUV (LightingUtil.hlsl:216-225); .xy only.
__device__ __forceinline__ void world_to_sky_uv(f3 c, float& u, float& v) {
    float ux = atan2f(c.z, c.x);
    float uy = asinf(c.y);
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
    int i = (int)f % n;
    return i < 0 ? i + n : i;
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
    float4 t00 = env[y0 * w + x0], t10 = env[y0 * w + x1];
    float4 t01 = env[y1 * w + x0], t11 = env[y1 * w + x1];
    return mk3(hlerp(hlerp(t00.x, t10.x, fx), hlerp(t01.x, t11.x, fx), fy),
               hlerp(hlerp(t00.y, t10.y, fx), hlerp(t01.y, t11.y, fx), fy),
               hlerp(hlerp(t00.z, t10.z, fx), hlerp(t01.z, t11.z, fx), fy));
}

}  // namespace pbr
