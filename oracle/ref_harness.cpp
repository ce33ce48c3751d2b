// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.  Built into oracle/_ref/libpbr_ref.so by
// oracle/Makefile, and only where /root/reference exists (the build container). The built library reads
// nothing from /root/reference at run time; it travels with the tree and serves bench.py's CPU baseline
// (kind "reference"). Stateless: every entry point may run concurrently on disjoint row bands.
//
// The reference's own light/BRDF code -- /root/reference/Source/Shaders/LightingUtil.hlsl, included
// UNMODIFIED by absolute path -- compiled as C++ on top of hlsl_prelude.hpp. It is included once
// per light-count permutation (the NUM_*_LIGHTS defines of Core.hlsl:1-12) so that the reference's
// ComputeLighting (LightingUtil.hlsl:170-200) runs as shipped whenever the counts match a
// permutation; other counts (beyond MAX_LIGHTS = 16, LightingUtil.hlsl:7) loop over the reference's
// ComputeDirectionalLight / ComputePointLight / ComputeSpotLight in ComputeLighting's order.
//
// The pixel-shader composition (Default.hlsl:47-161: V, F0 resolve, ambient, tonemap, gamma) needs
// texture/cbuffer syntax g++ cannot take, so those ~12 lines are restated below, each citing its line.
// Output: golden vectors (tests/golden/gen_golden.py) that pin oracle/pbr_oracle.c.
#include <cstdint>
#include <cstddef>
#include <cmath>

#include "hlsl_prelude.hpp"
#include "pbr_oracle.h"

#define PBR_REF_LIGHTINGUTIL "/root/reference/Source/Shaders/LightingUtil.hlsl"

namespace hlsl {
// Reference scene permutation: Core.hlsl defaults (4 directional, 0 point, 0 spot).
namespace ref_d4 {
#define NUM_DIR_LIGHTS 4
#define NUM_POINT_LIGHTS 0
#define NUM_SPOT_LIGHTS 0
#include PBR_REF_LIGHTINGUTIL
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS
}  // namespace ref_d4
namespace ref_p1 {
#define NUM_DIR_LIGHTS 0
#define NUM_POINT_LIGHTS 1
#define NUM_SPOT_LIGHTS 0
#include PBR_REF_LIGHTINGUTIL
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS
}  // namespace ref_p1
namespace ref_p8 {
#define NUM_DIR_LIGHTS 0
#define NUM_POINT_LIGHTS 8
#define NUM_SPOT_LIGHTS 0
#include PBR_REF_LIGHTINGUTIL
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS
}  // namespace ref_p8
namespace ref_mix {
#define NUM_DIR_LIGHTS 4
#define NUM_POINT_LIGHTS 8
#define NUM_SPOT_LIGHTS 4
#include PBR_REF_LIGHTINGUTIL
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS
}  // namespace ref_mix

// Linear-wrap bilinear filter over an R16G16B16A16_UNORM texture (the D3D sampler g_SamLinearWrap,
// PBRApp.cpp:1157-1162), in the fp32 form DESIGN.md fixes (hardware 8-bit sub-texel weights are not
// reproducible: texture filtering parity is defined by this formula, not pinned to a GPU).
struct Texture2D {
    const uint16_t* texels;
    int w, h;
    const float* ftexels = nullptr;  // RGBA fp32 texture (HDR, or UNORM16 pre-decoded), used if set
    static int wrap(float f, int n) {
        if (!(f == f) || f > 2.0e9f || f < -2.0e9f) return 0;
        int i = (int)f % n;
        return i < 0 ? i + n : i;
    }
    float fetch(int x, int y, int c) const {
        const size_t i = ((size_t)y * (size_t)w + (size_t)x) * 4u + (size_t)c;
        return ftexels ? ftexels[i] : (float)texels[i] / 65535.0f;
    }
    float3 Sample(float3 uvw) const {  // only .xy is a coordinate (Default.hlsl:144)
        float x = uvw.x * (float)w - 0.5f, y = uvw.y * (float)h - 0.5f;
        float x0f = std::floor(x), y0f = std::floor(y);
        float fx = x - x0f, fy = y - y0f;
        int x0 = wrap(x0f, w), y0 = wrap(y0f, h);
        int x1 = x0 + 1 == w ? 0 : x0 + 1, y1 = y0 + 1 == h ? 0 : y0 + 1;
        float r[3];
        for (int c = 0; c < 3; ++c)
            r[c] = lerp(lerp(fetch(x0, y0, c), fetch(x1, y0, c), fx), lerp(fetch(x0, y1, c), fetch(x1, y1, c), fx), fy);
        return float3(r[0], r[1], r[2]);
    }
};
}  // namespace hlsl

using namespace hlsl;

namespace {

template <class Light>
void to_ref_light(const oracle_light& s, Light& d) {
    d.Strength = float3(s.strength[0], s.strength[1], s.strength[2]);
    d.SpotPower = s.spot_power;
    d.Direction = float3(s.direction[0], s.direction[1], s.direction[2]);
    d.__PAD000 = 0.0f;
    d.Position = float3(s.position[0], s.position[1], s.position[2]);
    d.__PAD001 = 0.0f;
}

// ComputeLighting through the reference permutation NS when the counts match it exactly.
template <int ND, int NP, int NS, class LightT, class MaterialT, class Fn>
bool try_permutation(const oracle_pass& ps, const oracle_light* lights, const MaterialT& mat, float3 pos,
                     float3 N, float3 V, float3& out, Fn compute_lighting) {
    if (ps.n_dir != ND || ps.n_point != NP || ps.n_spot != NS) return false;
    LightT g[16];
    for (int i = 0; i < ND + NP + NS; ++i) to_ref_light(lights[i], g[i]);
    out = compute_lighting(g, mat, pos, N, V, float3(1.0f));
    return true;
}

float3 direct_light(const oracle_pass& ps, const oracle_light* lights, const ref_d4::Material& mat, float3 pos,
                    float3 N, float3 V) {
    float3 r;
    if (try_permutation<4, 0, 0, ref_d4::Light>(ps, lights, mat, pos, N, V, r, ref_d4::ComputeLighting)) return r;
    {
        ref_p1::Material m1 = {mat.DiffuseAlbedo, mat.Metallic, mat.FresnelR0, mat.Roughness, mat.Transmission,
                               mat.Opacity, mat.Emissive, mat.Sheen, mat.ClearCoatThickness, mat.ClearCoatRoughness,
                               mat.Anisotropy, mat.AnisotropyRotation};
        if (try_permutation<0, 1, 0, ref_p1::Light>(ps, lights, m1, pos, N, V, r, ref_p1::ComputeLighting)) return r;
        ref_p8::Material m8 = {mat.DiffuseAlbedo, mat.Metallic, mat.FresnelR0, mat.Roughness, mat.Transmission,
                               mat.Opacity, mat.Emissive, mat.Sheen, mat.ClearCoatThickness, mat.ClearCoatRoughness,
                               mat.Anisotropy, mat.AnisotropyRotation};
        if (try_permutation<0, 8, 0, ref_p8::Light>(ps, lights, m8, pos, N, V, r, ref_p8::ComputeLighting)) return r;
        ref_mix::Material mm = {mat.DiffuseAlbedo, mat.Metallic, mat.FresnelR0, mat.Roughness, mat.Transmission,
                                mat.Opacity, mat.Emissive, mat.Sheen, mat.ClearCoatThickness, mat.ClearCoatRoughness,
                                mat.Anisotropy, mat.AnisotropyRotation};
        if (try_permutation<4, 8, 4, ref_mix::Light>(ps, lights, mm, pos, N, V, r, ref_mix::ComputeLighting)) return r;
    }
    // Any other count: ComputeLighting's three loops (LightingUtil.hlsl:176-199) over the reference's
    // per-light functions, same order, same `result +=`, same shadowFactor multiply on directional lights.
    float3 result = 0.0f;
    float3 shadowFactor = 1.0f;
    int i = 0;
    ref_d4::Light L;
    for (i = 0; i < ps.n_dir; i++) {
        to_ref_light(lights[i], L);
        result += shadowFactor * ref_d4::ComputeDirectionalLight(L, mat, N, V);
    }
    for (i = ps.n_dir; i < ps.n_dir + ps.n_point; i++) {
        to_ref_light(lights[i], L);
        result += ref_d4::ComputePointLight(L, mat, pos, N, V);
    }
    for (i = ps.n_dir + ps.n_point; i < ps.n_dir + ps.n_point + ps.n_spot; i++) {
        to_ref_light(lights[i], L);
        result += ref_d4::ComputeSpotLight(L, mat, pos, N, V);
    }
    return result;
}

}  // namespace

namespace {

// PS (Default.hlsl:47-161) for one G-buffer pixel.
float4 ps_pixel(const float* const* planes, int64_t i, const oracle_pass& ps, const oracle_light* lights,
                const Texture2D& env) {
    float3 PosW(planes[ORACLE_PX][i], planes[ORACLE_PY][i], planes[ORACLE_PZ][i]);
    float3 N(planes[ORACLE_NX][i], planes[ORACLE_NY][i], planes[ORACLE_NZ][i]);
    float3 g_CameraPosW(ps.eye[0], ps.eye[1], ps.eye[2]);
    // Default.hlsl:53
    float3 V = normalize(g_CameraPosW - PosW);
    float3 diffuseAlbedo(planes[ORACLE_AR][i], planes[ORACLE_AG][i], planes[ORACLE_AB][i]);
    float metallic = planes[ORACLE_METAL][i];
    float roughness = planes[ORACLE_ROUGH][i];
    float3 F0;
    if (ps.use_f0_plane) {  // Default.hlsl:92
        F0 = float3(planes[ORACLE_F0R][i], planes[ORACLE_F0G][i], planes[ORACLE_F0B][i]);
    } else {  // Default.hlsl:94-95
        F0 = float3(ps.fresnel_r0[0], ps.fresnel_r0[1], ps.fresnel_r0[2]);
        F0 = lerp(F0, diffuseAlbedo, metallic);
    }
    // Default.hlsl:121-133 (only the first four members are read by the BRDF)
    ref_d4::Material mat = {diffuseAlbedo, metallic, F0, roughness, float3(1.0f), ps.opacity,
                            float3(0.0f), 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    // Default.hlsl:135-137
    float3 directLight = direct_light(ps, lights, mat, PosW, N, V);
    float3 ambient;
    if (ps.ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE) {
        // Default.hlsl:141-146 (the commented-out IBL block)
        float3 kS = ref_d4::FresnelSchlick(N, V, F0);
        float3 kD = 1.0f - kS;
        kD *= (1.0f - metallic);
        float3 irradiance = env.Sample(ref_d4::WorldToSkyUV(N));
        float3 diffuse = irradiance * diffuseAlbedo;
        ambient = (kD * diffuse);
    } else {
        // Default.hlsl:150  g_AmbientLight * diffuseAlbedo
        float4 g_AmbientLight{ps.ambient[0], ps.ambient[1], ps.ambient[2], 1.0f};
        ambient = g_AmbientLight.rgb() * diffuseAlbedo;
    }
    if (ps.apply_ao) ambient = ambient * planes[ORACLE_AO][i];  // extension, off in the reference
    float3 litColor = ambient + directLight;
    // Default.hlsl:153, 155
    litColor = litColor / (litColor + float3(1.0f, 1.0f, 1.0f));
    litColor = pow(litColor, (1.0f / 2.2f));
    return float4{litColor.x, litColor.y, litColor.z, ps.opacity};  // Default.hlsl:160
}

// Skybox.hlsl:41-49 (PS) for one background pixel; PosW = the G-buffer normal planes.
float4 sky_pixel(const float* const* planes, int64_t i, const Texture2D& sky) {
    float3 PosW(planes[ORACLE_NX][i], planes[ORACLE_NY][i], planes[ORACLE_NZ][i]);
    float3 sampleCoord = normalize(PosW);
    sampleCoord = ref_d4::WorldToSkyUV(sampleCoord);
    float3 skyColor = sky.Sample(sampleCoord);
    skyColor = skyColor / (skyColor + float3(1.0f, 1.0f, 1.0f));
    skyColor = pow(skyColor, (1.0f / 2.2f));
    return float4{skyColor.x, skyColor.y, skyColor.z, 1.0f};
}

uint8_t unorm8(float c) {  // D3D FLOAT -> UNORM (the R8G8B8A8_UNORM back buffer, d3dApp.h:124)
    if (!(c == c)) return 0;
    c = c > 1.0f ? 1.0f : c;
    c = c < 0.0f ? 0.0f : c;
    return (uint8_t)(c * 255.0f + 0.5f);
}

}  // namespace

extern "C" int ref_shade_frame(int width, int height, int64_t stride, const float* const* planes,
                               const oracle_pass* pass, const oracle_light* lights, const oracle_frame* frame,
                               void* out, int64_t out_stride, int /*n_threads*/) {
    if (!planes || !pass || !frame || !out || width < 0 || height < 0) return -1;
    if (pass->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE && !frame->env_rgba) return -1;
    if (frame->coverage && !frame->sky_rgba) return -1;
    Texture2D env{nullptr, frame->env_w, frame->env_h, frame->env_rgba};
    Texture2D sky{nullptr, frame->sky_w, frame->sky_h, frame->sky_rgba};
    for (int y = 0; y < height; ++y) {
        for (int x = 0; x < width; ++x) {
            const int64_t i = (int64_t)y * stride + x;
            const bool background = frame->coverage && frame->coverage[(int64_t)y * frame->coverage_stride + x] == 0;
            const float4 c = background ? sky_pixel(planes, i, sky) : ps_pixel(planes, i, *pass, lights, env);
            const int64_t off = ((int64_t)y * out_stride + x) * 4;
            if (frame->format == ORACLE_OUTPUT_RGBA8) {
                uint8_t* o = static_cast<uint8_t*>(out) + off;
                o[0] = unorm8(c.x); o[1] = unorm8(c.y); o[2] = unorm8(c.z); o[3] = unorm8(c.w);
            } else {
                float* o = static_cast<float*>(out) + off;
                o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = c.w;
            }
        }
    }
    return 0;
}

extern "C" int ref_shade(int width, int height, int64_t stride, const float* const* planes, const oracle_pass* pass,
                         const oracle_light* lights, const uint16_t* env_rgba16, int env_w, int env_h, float* out,
                         int64_t out_stride, int /*n_threads*/) {
    if (!planes || !pass || !out || width < 0 || height < 0) return -1;
    if (pass->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE && !env_rgba16) return -1;
    Texture2D env{env_rgba16, env_w, env_h};
    for (int y = 0; y < height; ++y) {
        for (int x = 0; x < width; ++x) {
            const float4 c = ps_pixel(planes, (int64_t)y * stride + x, *pass, lights, env);
            float* o = out + ((int64_t)y * out_stride + x) * 4;
            o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = c.w;
        }
    }
    return 0;
}
