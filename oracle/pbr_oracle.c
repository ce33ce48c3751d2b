/*
 * oracle/pbr_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the reference's per-pixel Cook-Torrance shading, written from
 *   /root/reference/Source/Shaders/Default.hlsl:47-161   (PS)
 *   /root/reference/Source/Shaders/LightingUtil.hlsl:35-225
 * in HLSL fp32 semantics (the "canonical fp32 semantics" of DESIGN.md):
 *   - every literal and every intermediate is fp32 (HLSL has no implicit double promotion);
 *   - no FMA contraction (build with -ffp-contract=off), IEEE division and sqrt;
 *   - dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z, normalize(v) = v / sqrt(dot(v,v));
 *   - max = IEEE maxNum (D3D10+: a NaN operand yields the other one), saturate(NaN) = 0;
 *   - lerp(x,y,s) = x + s*(y-x); pow/atan2/asin from libm.
 * Parity pin: the fixtures in tests/golden/ were produced by oracle/_ref (the reference's own LightingUtil.hlsl
 * compiled as C++), and tests/test_oracle_golden.py requires bit equality with them.
 */
#include "pbr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stddef.h>
#include <stdlib.h>

typedef struct { float x, y, z; } v3;

static inline v3 v3make(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float hmax(float a, float b) { return fmaxf(a, b); }
static inline float hsat(float a) { return fminf(fmaxf(a, 0.0f), 1.0f); }
static inline v3 norm3(v3 v) {
    float s = sqrtf(dot3(v, v));
    return v3make(v.x / s, v.y / s, v.z / s);
}

/* The HLSL literal 3.14159265359 in fp32 (LightingUtil.hlsl:59, 103). */
static const float kPi = 3.14159265359f;

typedef struct {
    v3 albedo;       /* Material.DiffuseAlbedo */
    float metallic;  /* Material.Metallic */
    v3 f0;           /* Material.FresnelR0 */
    float roughness; /* Material.Roughness */
} mat_t;

/* CalcAttenuation, LightingUtil.hlsl:35-40 */
static inline float calc_attenuation(float d) {
    float dsat = hmax(d, 0.01f);
    return 1.0f / (dsat * dsat);
}

/* FresnelSchlick, LightingUtil.hlsl:43-47 */
static inline v3 fresnel_schlick(v3 h, v3 v, v3 f0) {
    float cos_theta = hsat(dot3(h, v));
    float p = powf(1.0f - cos_theta, 5.0f);
    return v3make(f0.x + (1.0f - f0.x) * p, f0.y + (1.0f - f0.y) * p, f0.z + (1.0f - f0.z) * p);
}

/* DistributionGGX, LightingUtil.hlsl:49-62 */
static inline float distribution_ggx(v3 n, v3 h, float roughness) {
    roughness = hmax(roughness, 0.05f);
    float a = roughness * roughness;
    float a_sqr = a * a;
    float n_dot_h = hmax(dot3(n, h), 0.0f);
    float n_dot_h_sqr = n_dot_h * n_dot_h;
    float nom = a_sqr;
    float denom = (n_dot_h_sqr * (a_sqr - 1.0f) + 1.0f);
    denom = kPi * denom * denom;
    return nom / denom;
}

/* GeometrySchlickGGX, LightingUtil.hlsl:64-73 (k from the unclamped roughness) */
static inline float geometry_schlick_ggx(float n_dot_v, float roughness) {
    float r = (roughness + 1.0f);
    float k = (r * r) / 8.0f;
    float nom = n_dot_v;
    float denom = n_dot_v * (1.0f - k) + k;
    return nom / denom;
}

/* GeometrySmith, LightingUtil.hlsl:75-83 */
static inline float geometry_smith(v3 n, v3 v, v3 l, float roughness) {
    float n_dot_v = hmax(dot3(n, v), 0.0f);
    float n_dot_l = hmax(dot3(n, l), 0.0f);
    float ggx2 = geometry_schlick_ggx(n_dot_v, roughness);
    float ggx1 = geometry_schlick_ggx(n_dot_l, roughness);
    return ggx1 * ggx2;
}

/* BRDFCookTorrance, LightingUtil.hlsl:85-104 */
static inline v3 brdf_cook_torrance(const mat_t* m, v3 radiance, v3 n, v3 v, v3 l, v3 h) {
    float ndf = distribution_ggx(n, h, m->roughness);
    float g = geometry_smith(n, v, l, m->roughness);
    v3 f = fresnel_schlick(h, v, m->f0);

    float ndf_g = ndf * g; /* NDF * G * F  evaluates (NDF*G)*F */
    v3 nom = v3make(ndf_g * f.x, ndf_g * f.y, ndf_g * f.z);
    float denom = 4.0f * hmax(dot3(n, v), 0.0f) * hmax(dot3(n, l), 0.0f) + 0.001f;
    v3 spec = v3make(nom.x / denom, nom.y / denom, nom.z / denom);

    v3 kd = v3make(1.0f - f.x, 1.0f - f.y, 1.0f - f.z);
    float one_minus_metal = 1.0f - m->metallic;
    kd.x *= one_minus_metal;
    kd.y *= one_minus_metal;
    kd.z *= one_minus_metal;

    float n_dot_l = hmax(dot3(n, l), 0.0f);
    v3 r;
    r.x = ((kd.x * m->albedo.x) / kPi + spec.x) * radiance.x * n_dot_l;
    r.y = ((kd.y * m->albedo.y) / kPi + spec.y) * radiance.y * n_dot_l;
    r.z = ((kd.z * m->albedo.z) / kPi + spec.z) * radiance.z * n_dot_l;
    return r;
}

static inline v3 lv_strength(const oracle_light* L) { return v3make(L->strength[0], L->strength[1], L->strength[2]); }
static inline v3 lv_direction(const oracle_light* L) { return v3make(L->direction[0], L->direction[1], L->direction[2]); }
static inline v3 lv_position(const oracle_light* L) { return v3make(L->position[0], L->position[1], L->position[2]); }

/* ComputeDirectionalLight, LightingUtil.hlsl:109-119 */
static inline v3 compute_directional(const oracle_light* light, const mat_t* m, v3 n, v3 v) {
    v3 d = lv_direction(light);
    v3 l = v3make(-d.x, -d.y, -d.z);
    v3 h = norm3(v3make(v.x + l.x, v.y + l.y, v.z + l.z));
    return brdf_cook_torrance(m, lv_strength(light), n, v, l, h);
}

/* ComputePointLight, LightingUtil.hlsl:124-142 ; spot variant 147-167 */
static inline v3 compute_point_or_spot(const oracle_light* light, const mat_t* m, v3 pos, v3 n, v3 v,
                                       int is_spot) {
    v3 lp = lv_position(light);
    v3 l = v3make(lp.x - pos.x, lp.y - pos.y, lp.z - pos.z);
    float d = sqrtf(dot3(l, l));
    if (d > 100.0f) return v3make(0.0f, 0.0f, 0.0f); /* range test, LightingUtil.hlsl:131 */
    l = v3make(l.x / d, l.y / d, l.z / d);
    v3 h = norm3(v3make(v.x + l.x, v.y + l.y, v.z + l.z));
    float att = calc_attenuation(d);
    if (is_spot) { /* LightingUtil.hlsl:163 */
        v3 dir = lv_direction(light);
        v3 nl = v3make(-l.x, -l.y, -l.z);
        att *= powf(hmax(dot3(nl, dir), 0.0f), light->spot_power);
    }
    v3 s = lv_strength(light);
    v3 radiance = v3make(s.x * att, s.y * att, s.z * att);
    return brdf_cook_torrance(m, radiance, n, v, l, h);
}

/* WorldToSkyUV, LightingUtil.hlsl:216-225 (only .xy is used as a texture coordinate) */
static inline void world_to_sky_uv(v3 c, float* u, float* v) {
    float ux = atan2f(c.z, c.x);
    float uy = asinf(c.y);
    ux = ux * 0.1591f;
    uy = uy * 0.3183f;
    ux = ux + 0.5f;
    uy = uy + 0.5f;
    uy = 1.0f - uy;
    ux = 1.0f - ux;
    ux = ux + 0.25f;
    *u = ux;
    *v = uy;
}

/* Linear-wrap bilinear sample (g_SamLinearWrap, PBRApp.cpp:1157-1162) of an RGBA fp32 texture: an
 * R16G16B16A16_UNORM texture is decoded once to u16 / 65535 (oracle_decode_unorm16); an HDR texture
 * is used as given. */
static inline int wrap_index(float f, int n) {
    if (!(f == f) || f > 2.0e9f || f < -2.0e9f) return 0; /* NaN coordinate: weights are NaN anyway */
    int i = (int)f % n;
    return i < 0 ? i + n : i;
}
static inline float texel(const float* env, int w, int x, int y, int c) {
    return env[((size_t)y * (size_t)w + (size_t)x) * 4u + (size_t)c];
}
static inline float lerpf_h(float a, float b, float t) { return a + t * (b - a); }
static v3 sample_linear_wrap(const float* env, int w, int h, float u, float v) {
    float x = u * (float)w - 0.5f;
    float y = v * (float)h - 0.5f;
    float x0f = floorf(x), y0f = floorf(y);
    float fx = x - x0f, fy = y - y0f;
    int x0 = wrap_index(x0f, w), y0 = wrap_index(y0f, h);
    int x1 = x0 + 1 == w ? 0 : x0 + 1;
    int y1 = y0 + 1 == h ? 0 : y0 + 1;
    float r[3];
    for (int c = 0; c < 3; ++c) {
        float t00 = texel(env, w, x0, y0, c), t10 = texel(env, w, x1, y0, c);
        float t01 = texel(env, w, x0, y1, c), t11 = texel(env, w, x1, y1, c);
        r[c] = lerpf_h(lerpf_h(t00, t10, fx), lerpf_h(t01, t11, fx), fy);
    }
    return v3make(r[0], r[1], r[2]);
}

typedef struct {
    int width, row0, row1;
    int64_t stride, out_stride;
    const float* const* planes;
    const oracle_pass* pass;
    const oracle_light* lights;
    const float* env;
    int env_w, env_h;
    const float* sky;
    int sky_w, sky_h;
    const uint8_t* coverage;
    int64_t coverage_stride;
    int format;
    void* out_any;
} job_t;

/* PS, Default.hlsl:47-161, one pixel. N is the already-resolved G-buffer normal (lines 50, 104-109
 * belong to the G-buffer fill). Returns 0 when the ALPHA_TEST permutation's clip discards the pixel
 * (its output is then left as it was). */
static int shade_pixel(const job_t* j, int64_t idx, float* o) {
    const float* const* P = j->planes;
    const oracle_pass* ps = j->pass;
    /* fragOpacity: the opacity map under ALPHA_TEST, clip(fragOpacity - 0.1f) (discard when negative;
     * NaN is not), else g_Opacity -- Default.hlsl:111-116 */
    float frag_opacity = ps->opacity;
    if (ps->alpha_test) {
        frag_opacity = P[ORACLE_OPACITY][idx];
        if (frag_opacity - 0.1f < 0.0f) return 0;
    }
    v3 pos = v3make(P[ORACLE_PX][idx], P[ORACLE_PY][idx], P[ORACLE_PZ][idx]);
    v3 n = v3make(P[ORACLE_NX][idx], P[ORACLE_NY][idx], P[ORACLE_NZ][idx]);
    /* V = normalize(g_CameraPosW - pin.PosW), Default.hlsl:53 */
    v3 v = norm3(v3make(ps->eye[0] - pos.x, ps->eye[1] - pos.y, ps->eye[2] - pos.z));

    mat_t m;
    m.albedo = v3make(P[ORACLE_AR][idx], P[ORACLE_AG][idx], P[ORACLE_AB][idx]);
    m.metallic = P[ORACLE_METAL][idx];
    m.roughness = P[ORACLE_ROUGH][idx];
    if (ps->use_f0_plane) { /* Default.hlsl:92 */
        m.f0 = v3make(P[ORACLE_F0R][idx], P[ORACLE_F0G][idx], P[ORACLE_F0B][idx]);
    } else { /* F0 = lerp(g_FresnelR0, diffuseAlbedo, metallic), Default.hlsl:94-95 */
        m.f0.x = lerpf_h(ps->fresnel_r0[0], m.albedo.x, m.metallic);
        m.f0.y = lerpf_h(ps->fresnel_r0[1], m.albedo.y, m.metallic);
        m.f0.z = lerpf_h(ps->fresnel_r0[2], m.albedo.z, m.metallic);
    }

    /* ComputeLighting, LightingUtil.hlsl:170-200: in-order sum from 0 */
    v3 direct = v3make(0.0f, 0.0f, 0.0f);
    int i = 0;
    for (; i < ps->n_dir; ++i) {
        v3 c = compute_directional(&j->lights[i], &m, n, v);
        /* shadowFactor (1,1,1) * c, LightingUtil.hlsl:181 */
        direct.x += 1.0f * c.x;
        direct.y += 1.0f * c.y;
        direct.z += 1.0f * c.z;
    }
    for (; i < ps->n_dir + ps->n_point; ++i) {
        v3 c = compute_point_or_spot(&j->lights[i], &m, pos, n, v, 0);
        direct.x += c.x; direct.y += c.y; direct.z += c.z;
    }
    for (; i < ps->n_dir + ps->n_point + ps->n_spot; ++i) {
        v3 c = compute_point_or_spot(&j->lights[i], &m, pos, n, v, 1);
        direct.x += c.x; direct.y += c.y; direct.z += c.z;
    }

    v3 ambient;
    if (ps->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE) {
        /* Default.hlsl:141-146 (commented-out IBL block, revived) */
        v3 ks = fresnel_schlick(n, v, m.f0);
        v3 kd = v3make(1.0f - ks.x, 1.0f - ks.y, 1.0f - ks.z);
        float om = 1.0f - m.metallic;
        kd.x *= om; kd.y *= om; kd.z *= om;
        float su, sv;
        world_to_sky_uv(n, &su, &sv);
        v3 irr = sample_linear_wrap(j->env, j->env_w, j->env_h, su, sv);
        v3 diffuse = v3make(irr.x * m.albedo.x, irr.y * m.albedo.y, irr.z * m.albedo.z);
        ambient = v3make(kd.x * diffuse.x, kd.y * diffuse.y, kd.z * diffuse.z);
    } else {
        /* g_AmbientLight * diffuseAlbedo (float4*float3 -> .rgb), Default.hlsl:150 */
        ambient = v3make(ps->ambient[0] * m.albedo.x, ps->ambient[1] * m.albedo.y, ps->ambient[2] * m.albedo.z);
    }
    if (ps->apply_ao) {
        float ao = P[ORACLE_AO][idx];
        ambient = v3make(ambient.x * ao, ambient.y * ao, ambient.z * ao);
    }
    v3 lit = v3make(ambient.x + direct.x, ambient.y + direct.y, ambient.z + direct.z);
    /* Reinhard, Default.hlsl:153 */
    lit = v3make(lit.x / (lit.x + 1.0f), lit.y / (lit.y + 1.0f), lit.z / (lit.z + 1.0f));
    /* gamma, Default.hlsl:155 */
    const float inv_gamma = 1.0f / 2.2f;
    o[0] = powf(lit.x, inv_gamma);
    o[1] = powf(lit.y, inv_gamma);
    o[2] = powf(lit.z, inv_gamma);
    o[3] = frag_opacity; /* Default.hlsl:160 */
    return 1;
}

/* The sky pass for a background pixel, Skybox.hlsl:37-49: sampleCoord = normalize(PosW) (the sky
 * dome's interpolated local position, here the G-buffer normal planes), WorldToSkyUV, sample
 * g_SkyArray[0] with linear-wrap, Reinhard, gamma, alpha 1. */
static void sky_pixel(const job_t* j, int64_t idx, float* o) {
    const float* const* P = j->planes;
    v3 c = norm3(v3make(P[ORACLE_NX][idx], P[ORACLE_NY][idx], P[ORACLE_NZ][idx]));
    float su, sv;
    world_to_sky_uv(c, &su, &sv);
    v3 col = sample_linear_wrap(j->sky, j->sky_w, j->sky_h, su, sv);
    col = v3make(col.x / (col.x + 1.0f), col.y / (col.y + 1.0f), col.z / (col.z + 1.0f));
    const float inv_gamma = 1.0f / 2.2f;
    o[0] = powf(col.x, inv_gamma);
    o[1] = powf(col.y, inv_gamma);
    o[2] = powf(col.z, inv_gamma);
    o[3] = 1.0f;
}

/* D3D FLOAT -> UNORM8 (the R8G8B8A8_UNORM back buffer, d3dApp.h:124; D3D11 functional spec
 * "FLOAT -> UNORM"): NaN -> 0; clamp to [0, 1]; c * 255 + 0.5 in fp32; truncate. */
uint8_t oracle_unorm8(float c) {
    if (!(c == c)) return 0;
    c = c > 1.0f ? 1.0f : c;
    c = c < 0.0f ? 0.0f : c;
    return (uint8_t)(c * 255.0f + 0.5f);
}

static void* run_rows(void* arg) {
    const job_t* j = (const job_t*)arg;
    for (int y = j->row0; y < j->row1; ++y) {
        for (int x = 0; x < j->width; ++x) {
            const int64_t idx = (int64_t)y * j->stride + x;
            const int64_t off = (int64_t)y * j->out_stride + x;
            float px[4];
            if (j->coverage && j->coverage[(int64_t)y * j->coverage_stride + x] == 0)
                sky_pixel(j, idx, px);
            else if (!shade_pixel(j, idx, px))
                continue; /* clip: the render target keeps its value */
            if (j->format == ORACLE_OUTPUT_RGBA8) {
                uint8_t* o8 = (uint8_t*)j->out_any + off * 4;
                for (int c = 0; c < 4; ++c) o8[c] = oracle_unorm8(px[c]);
            } else {
                float* o = (float*)j->out_any + off * 4;
                for (int c = 0; c < 4; ++c) o[c] = px[c];
            }
        }
    }
    return NULL;
}

void oracle_decode_unorm16(const uint16_t* src, int64_t n_values, float* dst) {
    for (int64_t i = 0; i < n_values; ++i) dst[i] = (float)src[i] / 65535.0f; /* R16G16B16A16_UNORM */
}

int oracle_shade_frame(int width, int height, int64_t stride, const float* const* planes, const oracle_pass* pass,
                       const oracle_light* lights, const oracle_frame* frame, void* out, int64_t out_stride,
                       int n_threads) {
    if (width < 0 || height < 0 || !planes || !pass || !frame || !out) return -1;
    if (stride < width || out_stride < width) return -1;
    if (frame->format != ORACLE_OUTPUT_RGBA32F && frame->format != ORACLE_OUTPUT_RGBA8) return -1;
    if (pass->n_dir < 0 || pass->n_point < 0 || pass->n_spot < 0) return -1;
    if (pass->n_dir + pass->n_point + pass->n_spot > 0 && !lights) return -1;
    if (pass->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE &&
        (!frame->env_rgba || frame->env_w <= 0 || frame->env_h <= 0)) return -1;
    if (frame->coverage && (!frame->sky_rgba || frame->sky_w <= 0 || frame->sky_h <= 0 ||
                            frame->coverage_stride < width)) return -1;
    for (int p = 0; p < ORACLE_AO; ++p)
        if (!planes[p]) return -1;
    if (pass->apply_ao && !planes[ORACLE_AO]) return -1;
    if (pass->use_f0_plane && (!planes[ORACLE_F0R] || !planes[ORACLE_F0G] || !planes[ORACLE_F0B])) return -1;
    if (pass->alpha_test && !planes[ORACLE_OPACITY]) return -1;
    if (width == 0 || height == 0) return 0;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > height) n_threads = height;
    if (n_threads > 256) n_threads = 256;

    job_t jobs[256];
    pthread_t th[256];
    for (int t = 0; t < n_threads; ++t) {
        job_t* j = &jobs[t];
        j->width = width;
        j->row0 = (int)((int64_t)height * t / n_threads);
        j->row1 = (int)((int64_t)height * (t + 1) / n_threads);
        j->stride = stride;
        j->out_stride = out_stride;
        j->planes = planes;
        j->pass = pass;
        j->lights = lights;
        j->env = frame->env_rgba;
        j->env_w = frame->env_w;
        j->env_h = frame->env_h;
        j->sky = frame->sky_rgba;
        j->sky_w = frame->sky_w;
        j->sky_h = frame->sky_h;
        j->coverage = frame->coverage;
        j->coverage_stride = frame->coverage_stride;
        j->format = frame->format;
        j->out_any = out;
    }
    if (n_threads == 1) {
        run_rows(&jobs[0]);
        return 0;
    }
    int started = 0;
    for (int t = 1; t < n_threads; ++t) {
        if (pthread_create(&th[t], NULL, run_rows, &jobs[t]) != 0) break;
        started = t;
    }
    for (int t = started + 1; t < n_threads; ++t) run_rows(&jobs[t]); /* threads that failed to start */
    run_rows(&jobs[0]);
    for (int t = 1; t <= started; ++t) pthread_join(th[t], NULL);
    return 0;
}

int oracle_shade(int width, int height, int64_t stride, const float* const* planes,
                 const oracle_pass* pass, const oracle_light* lights,
                 const uint16_t* env_rgba16, int env_w, int env_h,
                 float* out, int64_t out_stride, int n_threads) {
    if (pass && pass->ambient_mode == ORACLE_AMBIENT_IBL_DIFFUSE && (!env_rgba16 || env_w <= 0 || env_h <= 0))
        return -1;
    oracle_frame fr = {0};
    float* env = NULL;
    if (env_rgba16 && env_w > 0 && env_h > 0) {
        const int64_t n = (int64_t)env_w * env_h * 4;
        env = (float*)malloc(sizeof(float) * (size_t)n);
        if (!env) return -2;
        oracle_decode_unorm16(env_rgba16, n, env);
        fr.env_rgba = env;
        fr.env_w = env_w;
        fr.env_h = env_h;
    }
    fr.format = ORACLE_OUTPUT_RGBA32F;
    const int rc = oracle_shade_frame(width, height, stride, planes, pass, lights, &fr, out, out_stride, n_threads);
    free(env);
    return rc;
}
