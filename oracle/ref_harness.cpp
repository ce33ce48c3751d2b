// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.  Built into oracle/_ref/libpbr_ref.so by
// oracle/Makefile, and only where /root/reference exists (the build container). The built library reads
// nothing from /root/reference at run time; it travels with the tree and serves bench.py's CPU baseline
// (kind "reference"). Entry points may run concurrently on disjoint row bands: all shader state
// (cbuffers, bound textures) is thread_local.
//
// What runs is the reference's own shader text:
//   * the pixel shader PS, Default.hlsl:47-161, with its includes Core.hlsl (cbuffers, resources) and
//     LightingUtil.hlsl (the BRDF, unmodified), after oracle/strip_hlsl.py's counted, syntax-only rewrite
//     (generated into oracle/_ref/gen/, never committed);
//   * the IBL_DIFFUSE ambient: the same PS with the author's commented-out block Default.hlsl:140-149
//     re-enabled (Default_ibl.hlsl, same script);
//   * the sky pass: Skybox.hlsl's PS (:37-49).
// The only restated shading code left is the AO extension (ps_pixel_ao_extension below): the reference
// has no AO term, so there is no reference text to compile for it.
//
// Permutations (the D3D_SHADER_MACRO defines of PBRApp.cpp:715-754): DIFFUSE/METALLIC/ROUGHNESS/NORMAL
// _TEXTURE = 1 with the G-buffer bound as the maps (ps_binding.inc explains the exact embedding),
// SPECULAR_TEXTURE = 1 for the F0 plane (config 4) else 0 (F0 = lerp(g_FresnelR0, albedo, metallic)),
// ALPHA_TEST = 0, and the ALPHA_TEST = 1 permutation of the same four (the reference's alphaTestedPS,
// PBRApp.cpp:750-765: the opacity map bound as the G-buffer's opacity plane; clip() in hlsl_prelude.hpp marks
// the pixel discarded and the harness leaves its output untouched). The light counts NUM_DIR/POINT/SPOT_LIGHTS (Core.hlsl:1-12) are compile-time in the
// reference; here they are runtime values behind macros whose preprocessor value is 1, so the
// `#if (NUM_*_LIGHTS > 0)` guards of ComputeLighting (LightingUtil.hlsl:178, 185, 192) keep their loops
// and each loop runs the pass's count (a loop with zero trips is what the #if removes). The shipped
// default permutation (Core.hlsl's own 4/0/0, no defines) is compiled too and runs whenever a pass has
// exactly those counts.
#include <cstdint>
#include <cstddef>
#include <cmath>

#include "hlsl_prelude.hpp"
#include "pbr_oracle.h"

#define PBR_HLSL_GLOBAL thread_local
#define PBR_ORACLE_MAX_LIGHTS 1024

namespace hlsl {

struct SamplerState {};

// A bound texture. Two kinds:
//  * constant: the G-buffer view of a material map -- Sample returns the pixel's stored value;
//  * bilinear: linear-wrap filtering over an RGBA texture (the sampler g_SamLinearWrap,
//    PBRApp.cpp:1157-1162), in the fp32 form DESIGN.md fixes (hardware 8-bit sub-texel weights are not
//    reproducible: texture-filtering parity is defined by this formula, not pinned to a GPU).
struct Texture2D {
    float4 value;
    const uint16_t* texels = nullptr;  // R16G16B16A16_UNORM texels (decoded as u16 / 65535)
    const float* ftexels = nullptr;    // RGBA fp32 texels (HDR, or UNORM16 pre-decoded), used if set
    int w = 0, h = 0;

    static Texture2D constant(float r, float g, float b, float a) {
        Texture2D t;
        t.value = float4(r, g, b, a);
        return t;
    }
    static int wrap(float f, int n) {
        if (!(f == f) || f > 2.0e9f || f < -2.0e9f) return 0;
        int i = (int)f % n;
        return i < 0 ? i + n : i;
    }
    float fetch(int x, int y, int c) const {
        const size_t i = ((size_t)y * (size_t)w + (size_t)x) * 4u + (size_t)c;
        return ftexels ? ftexels[i] : (float)texels[i] / 65535.0f;
    }
    float4 Sample(SamplerState, float2 uv) const {
        if (!texels && !ftexels) return value;
        float x = uv.x * (float)w - 0.5f, y = uv.y * (float)h - 0.5f;
        float x0f = std::floor(x), y0f = std::floor(y);
        float fx = x - x0f, fy = y - y0f;
        int x0 = wrap(x0f, w), y0 = wrap(y0f, h);
        int x1 = x0 + 1 == w ? 0 : x0 + 1, y1 = y0 + 1 == h ? 0 : y0 + 1;
        float r[4];
        for (int c = 0; c < 4; ++c)
            r[c] = lerp(lerp(fetch(x0, y0, c), fetch(x1, y0, c), fx), lerp(fetch(x0, y1, c), fetch(x1, y1, c), fx), fy);
        return float4(r[0], r[1], r[2], r[3]);
    }
};

template <class Light>
inline void pbr_to_ref_light(const oracle_light& s, Light& d) {
    d.Strength = float3(s.strength[0], s.strength[1], s.strength[2]);
    d.SpotPower = s.spot_power;
    d.Direction = float3(s.direction[0], s.direction[1], s.direction[2]);
    d.__PAD000 = 0.0f;
    d.Position = float3(s.position[0], s.position[1], s.position[2]);
    d.__PAD001 = 0.0f;
}

// Runtime light counts (see the header comment). In an #if the identifiers evaluate to 0, so
// PBR_RUNTIME_COUNT(n) is 1 there; in C++ it is n.
inline thread_local int pbr_num_dir = 0, pbr_num_point = 0, pbr_num_spot = 0;
constexpr int pbr_pp_one = 1;
#define PBR_RUNTIME_COUNT(n) ((n) + 1 - pbr_pp_one)

#define DIFFUSE_TEXTURE 1
#define METALLIC_TEXTURE 1
#define ROUGHNESS_TEXTURE 1
#define NORMAL_TEXTURE 1
#define ALPHA_TEST 0
#define DISPLACEMENT_TEXTURE 0

// Default.hlsl as shipped (constant ambient, Default.hlsl:150).
#define NUM_DIR_LIGHTS PBR_RUNTIME_COUNT(pbr_num_dir)
#define NUM_POINT_LIGHTS PBR_RUNTIME_COUNT(pbr_num_point)
#define NUM_SPOT_LIGHTS PBR_RUNTIME_COUNT(pbr_num_spot)
#define SPECULAR_TEXTURE 0
namespace ps_const {
#include "Default.hlsl"
#include "ps_binding.inc"
}  // namespace ps_const
namespace ps_ibl {
#include "Default_ibl.hlsl"
#include "ps_binding.inc"
}  // namespace ps_ibl
#undef SPECULAR_TEXTURE
#define SPECULAR_TEXTURE 1
namespace ps_const_f0map {
#include "Default.hlsl"
#include "ps_binding.inc"
}  // namespace ps_const_f0map
namespace ps_ibl_f0map {
#include "Default_ibl.hlsl"
#include "ps_binding.inc"
}  // namespace ps_ibl_f0map
#undef SPECULAR_TEXTURE
#undef ALPHA_TEST
#define ALPHA_TEST 1
#define SPECULAR_TEXTURE 0
namespace ps_const_at {
#include "Default.hlsl"
#include "ps_binding.inc"
}  // namespace ps_const_at
namespace ps_ibl_at {
#include "Default_ibl.hlsl"
#include "ps_binding.inc"
}  // namespace ps_ibl_at
#undef SPECULAR_TEXTURE
#define SPECULAR_TEXTURE 1
namespace ps_const_f0map_at {
#include "Default.hlsl"
#include "ps_binding.inc"
}  // namespace ps_const_f0map_at
namespace ps_ibl_f0map_at {
#include "Default_ibl.hlsl"
#include "ps_binding.inc"
}  // namespace ps_ibl_f0map_at
#undef SPECULAR_TEXTURE
#undef ALPHA_TEST
#define ALPHA_TEST 0
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS

// The shipped permutation: Core.hlsl:1-12 supplies its own 4 / 0 / 0 counts.
#define SPECULAR_TEXTURE 0
namespace ps_shipped {
#include "Default.hlsl"
#include "ps_binding.inc"
constexpr int kDir = NUM_DIR_LIGHTS, kPoint = NUM_POINT_LIGHTS, kSpot = NUM_SPOT_LIGHTS;
}  // namespace ps_shipped
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS

// Skybox.hlsl (its PS reads g_SkyArray[0] only; no light loop runs).
namespace sky {
#include "Skybox.hlsl"
}  // namespace sky
#undef NUM_DIR_LIGHTS
#undef NUM_POINT_LIGHTS
#undef NUM_SPOT_LIGHTS
#undef SPECULAR_TEXTURE

}  // namespace hlsl

using namespace hlsl;

namespace {

enum Variant { kShipped, kConst, kIbl, kConstF0, kIblF0, kConstAt, kIblAt, kConstF0At, kIblF0At };

Variant pick(const oracle_pass& ps) {
    const bool ibl = ps.ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE;
    if (ps.alpha_test) return ps.use_f0_plane ? (ibl ? kIblF0At : kConstF0At) : (ibl ? kIblAt : kConstAt);
    if (ps.use_f0_plane) return ibl ? kIblF0 : kConstF0;
    if (ibl) return kIbl;
    if (ps.n_dir == ps_shipped::kDir && ps.n_point == ps_shipped::kPoint && ps.n_spot == ps_shipped::kSpot)
        return kShipped;
    return kConst;
}

void bind(Variant v, const oracle_pass& ps, const oracle_light* lights, const Texture2D& env) {
    pbr_num_dir = ps.n_dir;
    pbr_num_point = ps.n_point;
    pbr_num_spot = ps.n_spot;
    switch (v) {
        case kShipped: ps_shipped::pbr_bind_pass(ps, lights, env); break;
        case kConst: ps_const::pbr_bind_pass(ps, lights, env); break;
        case kIbl: ps_ibl::pbr_bind_pass(ps, lights, env); break;
        case kConstF0: ps_const_f0map::pbr_bind_pass(ps, lights, env); break;
        case kIblF0: ps_ibl_f0map::pbr_bind_pass(ps, lights, env); break;
        case kConstAt: ps_const_at::pbr_bind_pass(ps, lights, env); break;
        case kIblAt: ps_ibl_at::pbr_bind_pass(ps, lights, env); break;
        case kConstF0At: ps_const_f0map_at::pbr_bind_pass(ps, lights, env); break;
        case kIblF0At: ps_ibl_f0map_at::pbr_bind_pass(ps, lights, env); break;
    }
    if (ps.apply_ao && v != kConst) ps_const::pbr_bind_pass(ps, lights, env);  // ps_pixel_ao_extension's
}

// Extension, not in the reference (the reference never reads its AO map): the same PS with
// the ambient term multiplied by the G-buffer AO. Restated line by line from Default.hlsl:47-161 on the
// compiled reference functions (ps_const / ps_ibl namespaces: ComputeLighting, FresnelSchlick,
// WorldToSkyUV, lerp); pbr_bind_pass must have run for the pass.
float4 ps_pixel_ao_extension(const float* const* planes, int64_t i, const oracle_pass& ps, const Texture2D& env) {
    float3 PosW(planes[ORACLE_PX][i], planes[ORACLE_PY][i], planes[ORACLE_PZ][i]);
    float3 N(planes[ORACLE_NX][i], planes[ORACLE_NY][i], planes[ORACLE_NZ][i]);
    float3 V = normalize(ps_const::cbPass::g_CameraPosW - PosW);                        // :53
    float3 diffuseAlbedo(planes[ORACLE_AR][i], planes[ORACLE_AG][i], planes[ORACLE_AB][i]);  // :80
    float metallic = planes[ORACLE_METAL][i];                                                 // :86
    float roughness = planes[ORACLE_ROUGH][i];                                                // :99
    float3 F0;
    if (ps.use_f0_plane) {
        F0 = float3(planes[ORACLE_F0R][i], planes[ORACLE_F0G][i], planes[ORACLE_F0B][i]);  // :92
    } else {
        F0 = float3(ps.fresnel_r0[0], ps.fresnel_r0[1], ps.fresnel_r0[2]);                  // :94
        F0 = lerp(F0, diffuseAlbedo, metallic);                                             // :95
    }
    float fragOpacity = ps.opacity;                                                        // :115
    if (ps.alpha_test) {                                                                    // :111-113
        fragOpacity = planes[ORACLE_OPACITY][i];
        clip(fragOpacity - 0.1f);
    }
    ps_const::Material mat = {diffuseAlbedo, metallic, F0, roughness, float3(1.0f), fragOpacity,
                              float3(0.0f), 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};                  // :121-133
    float3 shadowFactor = 1.0f;
    float3 directLight = ps_const::ComputeLighting(ps_const::cbPass::g_Lights, mat, PosW, N, V, shadowFactor);
    float3 ambient;
    if (ps.ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE) {  // :141-146
        float3 kS = ps_const::FresnelSchlick(N, V, F0);
        float3 kD = 1.0f - kS;
        kD *= (1.0f - metallic);
        float3 irradiance = env.Sample(SamplerState{}, ps_const::WorldToSkyUV(N)).rgb();
        float3 diffuse = irradiance * diffuseAlbedo;
        ambient = (kD * diffuse);
    } else {
        ambient = ps_const::cbPass::g_AmbientLight * diffuseAlbedo;  // :150
    }
    ambient = ambient * planes[ORACLE_AO][i];  // the extension
    float3 litColor = ambient + directLight;
    litColor = litColor / (litColor + float3(1.0f, 1.0f, 1.0f));  // :153
    litColor = pow(litColor, (1.0f / 2.2f));                      // :155
    return float4(litColor, fragOpacity);                         // :160
}

float4 shade_pixel(Variant v, const float* const* planes, int64_t i, const oracle_pass& ps, const Texture2D& env) {
    if (ps.apply_ao) return ps_pixel_ao_extension(planes, i, ps, env);
    switch (v) {
        case kShipped: return ps_shipped::pbr_shade_pixel(planes, i);
        case kConst: return ps_const::pbr_shade_pixel(planes, i);
        case kIbl: return ps_ibl::pbr_shade_pixel(planes, i);
        case kConstF0: return ps_const_f0map::pbr_shade_pixel(planes, i);
        case kIblF0: return ps_ibl_f0map::pbr_shade_pixel(planes, i);
        case kConstAt: return ps_const_at::pbr_shade_pixel(planes, i);
        case kIblAt: return ps_ibl_at::pbr_shade_pixel(planes, i);
        case kConstF0At: return ps_const_f0map_at::pbr_shade_pixel(planes, i);
        case kIblF0At: return ps_ibl_f0map_at::pbr_shade_pixel(planes, i);
    }
    return float4();
}

// Skybox.hlsl PS for one background pixel; the dome's interpolated local position (pin.PosW) is the
// G-buffer normal planes.
float4 sky_pixel(const float* const* planes, int64_t i) {
    sky::VertexOut pin;
    pin.PosW = float3(planes[ORACLE_NX][i], planes[ORACLE_NY][i], planes[ORACLE_NZ][i]);
    return sky::PS(pin);
}

uint8_t unorm8(float c) {  // D3D FLOAT -> UNORM (the R8G8B8A8_UNORM back buffer, d3dApp.h:124)
    if (!(c == c)) return 0;
    c = c > 1.0f ? 1.0f : c;
    c = c < 0.0f ? 0.0f : c;
    return (uint8_t)(c * 255.0f + 0.5f);
}

bool counts_ok(const oracle_pass& ps) {
    return ps.n_dir >= 0 && ps.n_point >= 0 && ps.n_spot >= 0 &&
           (int64_t)ps.n_dir + ps.n_point + ps.n_spot <= PBR_ORACLE_MAX_LIGHTS;
}
bool planes_ok(const float* const* planes, const oracle_pass& ps) { return !ps.alpha_test || planes[ORACLE_OPACITY]; }

}  // namespace

extern "C" int ref_shade_frame(int width, int height, int64_t stride, const float* const* planes,
                               const oracle_pass* pass, const oracle_light* lights, const oracle_frame* frame,
                               void* out, int64_t out_stride, int /*n_threads*/) {
    if (!planes || !pass || !frame || !out || width < 0 || height < 0 || !counts_ok(*pass) || !planes_ok(planes, *pass))
        return -1;
    if (pass->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE && !frame->env_rgba) return -1;
    if (frame->coverage && !frame->sky_rgba) return -1;
    Texture2D env, skytex;
    env.ftexels = frame->env_rgba, env.w = frame->env_w, env.h = frame->env_h;
    skytex.ftexels = frame->sky_rgba, skytex.w = frame->sky_w, skytex.h = frame->sky_h;
    const Variant v = pick(*pass);
    bind(v, *pass, lights, env);
    sky::g_SkyArray[0] = skytex;  // Core.hlsl:16, PBRApp.cpp:1205-1210
    for (int y = 0; y < height; ++y) {
        for (int x = 0; x < width; ++x) {
            const int64_t i = (int64_t)y * stride + x;
            const bool background = frame->coverage && frame->coverage[(int64_t)y * frame->coverage_stride + x] == 0;
            g_clip_discarded = false;
            const float4 c = background ? sky_pixel(planes, i) : shade_pixel(v, planes, i, *pass, env);
            if (g_clip_discarded) continue;  // clip(): the render target keeps its value
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
    if (!planes || !pass || !out || width < 0 || height < 0 || !counts_ok(*pass) || !planes_ok(planes, *pass)) return -1;
    if (pass->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE && !env_rgba16) return -1;
    Texture2D env;
    env.texels = env_rgba16, env.w = env_w, env.h = env_h;
    const Variant v = pick(*pass);
    bind(v, *pass, lights, env);
    for (int y = 0; y < height; ++y) {
        for (int x = 0; x < width; ++x) {
            g_clip_discarded = false;
            const float4 c = shade_pixel(v, planes, (int64_t)y * stride + x, *pass, env);
            if (g_clip_discarded) continue;  // clip(): the render target keeps its value
            float* o = out + ((int64_t)y * out_stride + x) * 4;
            o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = c.w;
        }
    }
    return 0;
}
