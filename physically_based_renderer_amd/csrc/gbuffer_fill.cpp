// gbuffer_fill.cpp -- host-side G-buffer fill for the benchmark scenes (pbr_gbuffer_fill,
// pbr_scene_pass in include/pbr/pbr_shade.h).
//
// This replaces the reference's rasteriser front-end (VS, Default.hlsl:22-45; the draw loop of
// PBRApp.cpp:1096-1135) with a flat structure-of-arrays fill on the CPU. Every value depends only on
// the pixel's global (x, y) and the scene seed, never on how rows are split across calls, threads or
// ranks, so a row band shaded on GPU r is bit-identical to the same rows of a single-GPU frame.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "pbr/pbr_shade.h"

namespace {

constexpr int kPosX = 0, kPosY = 1, kPosZ = 2, kNx = 3, kNy = 4, kNz = 5, kAr = 6, kAg = 7, kAb = 8, kMetal = 9,
              kRough = 10, kAo = 11, kF0r = 12, kF0g = 13, kF0b = 14;

inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Uniform [0, 1) with 24 random bits: exactly representable, identical on every host.
inline float u01(uint64_t seed, uint64_t index, uint32_t k) {
    return (float)(splitmix64(seed + index * 16u + k) >> 40) * (1.0f / 16777216.0f);
}

inline float lerp_h(float x, float y, float s) { return x + s * (y - x); }  // HLSL lerp

constexpr uint64_t kLightStream = 0x4C49474854535452ull;  // independent stream for light lists

struct Row {
    float* p[15];
    uint8_t* cov;  // coverage row (1 = geometry, 0 = background), or nullptr
};

inline void set_cov(Row r, int x, bool geometry) {
    if (r.cov) r.cov[x] = geometry ? 1 : 0;
}

void fill_random_covered(const pbr_scene_desc& sc, int y, Row r) {
    const pbr_scene_assets* as = sc.assets;
    const int S = as->rust_size;
    for (int x = 0; x < sc.width; ++x) {
        const uint64_t g = (uint64_t)y * (uint64_t)sc.width + (uint64_t)x;
        r.p[kPosX][x] = -10.0f + 20.0f * u01(sc.seed, g, 0);
        r.p[kPosY][x] = -10.0f + 20.0f * u01(sc.seed, g, 1);
        r.p[kPosZ][x] = 10.0f * u01(sc.seed, g, 2);
        float nx = 2.0f * u01(sc.seed, g, 3) - 1.0f, ny = 2.0f * u01(sc.seed, g, 4) - 1.0f,
              nz = 2.0f * u01(sc.seed, g, 5) - 1.0f;
        const float l2 = nx * nx + ny * ny + nz * nz;
        if (l2 < 1e-6f) {
            nx = 0.0f, ny = 1.0f, nz = 0.0f;
        } else {
            const float l = std::sqrt(l2);
            nx = nx / l, ny = ny / l, nz = nz / l;
        }
        r.p[kNx][x] = nx;
        r.p[kNy][x] = ny;
        r.p[kNz][x] = nz;
        const float ar = u01(sc.seed, g, 6), ag = u01(sc.seed, g, 7), ab = u01(sc.seed, g, 8);
        r.p[kAr][x] = ar;
        r.p[kAg][x] = ag;
        r.p[kAb][x] = ab;
        // rustediron metallic / roughness (PBRApp.cpp:1251-1255), tiled over the frame (wrap)
        const size_t t = (size_t)(y % S) * (size_t)S + (size_t)(x % S);
        const float metal = (float)as->rust_metallic[t] / 255.0f;
        r.p[kMetal][x] = metal;
        r.p[kRough][x] = (float)as->rust_roughness[t] / 255.0f;
        r.p[kAo][x] = 1.0f;
        // F0 plane = lerp(0.04, albedo, metallic) (Default.hlsl:94-95): an F0-plane pass over this
        // frame must equal the in-kernel metallic workflow bit for bit.
        r.p[kF0r][x] = lerp_h(0.04f, ar, metal);
        r.p[kF0g][x] = lerp_h(0.04f, ag, metal);
        r.p[kF0b][x] = lerp_h(0.04f, ab, metal);
    }
}

// Config 1: the reference camera (Camera(pi/4, w, h, 0.1, 100) at (0, 0, -5) looking +z, left-handed;
// PBRApp.cpp:652-659) ray-cast against the unit sphere at the origin (the rust sphere,
// PBRApp.cpp:1023-1027). UV = (theta / 2pi, phi / pi) as SphereMesh (Mesh.h:525-526).
int64_t fill_sphere(const pbr_scene_desc& sc, int y, Row r) {
    const pbr_scene_assets* as = sc.assets;
    const int S = as->rust_size;
    const double t = std::tan(M_PI / 8.0), aspect = (double)sc.width / (double)sc.height;
    int64_t covered = 0;
    for (int x = 0; x < sc.width; ++x) {
        double dx = (2.0 * (x + 0.5) / sc.width - 1.0) * t * aspect, dy = (1.0 - 2.0 * (y + 0.5) / sc.height) * t,
               dz = 1.0;
        const double il = 1.0 / std::sqrt(dx * dx + dy * dy + dz * dz);
        dx *= il, dy *= il, dz *= il;
        const double oz = -5.0;  // eye (0, 0, -5)
        const double b = oz * dz, c = oz * oz - 1.0, disc = b * b - c;
        set_cov(r, x, disc >= 0.0);
        if (disc >= 0.0) {
            ++covered;
            const double tt = -b - std::sqrt(disc);
            const double px = dx * tt, py = dy * tt, pz = oz + dz * tt;
            r.p[kPosX][x] = (float)px;
            r.p[kPosY][x] = (float)py;
            r.p[kPosZ][x] = (float)pz;
            const double nl = std::sqrt(px * px + py * py + pz * pz);
            r.p[kNx][x] = (float)(px / nl);
            r.p[kNy][x] = (float)(py / nl);
            r.p[kNz][x] = (float)(pz / nl);
            double u = std::atan2(pz, px) / (2.0 * M_PI);
            u -= std::floor(u);
            const double v = std::acos(std::fmin(std::fmax(py / nl, -1.0), 1.0)) / M_PI;
            const int tx = std::min(S - 1, (int)(u * S)), ty = std::min(S - 1, (int)(v * S));
            const size_t ti = (size_t)ty * S + tx;
            const float metal = (float)as->rust_metallic[ti] / 255.0f;
            r.p[kAr][x] = r.p[kAg][x] = r.p[kAb][x] = 0.5f;  // basecolor map missing from the snapshot
            r.p[kMetal][x] = metal;
            r.p[kRough][x] = (float)as->rust_roughness[ti] / 255.0f;
            r.p[kF0r][x] = r.p[kF0g][x] = r.p[kF0b][x] = lerp_h(0.04f, 0.5f, metal);
        } else {
            // Background: a far point on the view ray, black and rough; the normal planes carry the
            // view direction, i.e. the point of the camera-centred sky dome this pixel sees (the sky
            // pass samples it, Skybox.hlsl:22-24, 41).
            r.p[kPosX][x] = (float)(dx * 100.0);
            r.p[kPosY][x] = (float)(dy * 100.0);
            r.p[kPosZ][x] = (float)(oz + dz * 100.0);
            r.p[kNx][x] = (float)dx;
            r.p[kNy][x] = (float)dy;
            r.p[kNz][x] = (float)dz;
            r.p[kAr][x] = r.p[kAg][x] = r.p[kAb][x] = 0.0f;
            r.p[kMetal][x] = 0.0f;
            r.p[kRough][x] = 1.0f;
            r.p[kF0r][x] = r.p[kF0g][x] = r.p[kF0b][x] = 0.04f;
        }
        r.p[kAo][x] = 1.0f;
    }
    return covered;
}

// Config 4: the plane y = 0 seen from straight above; z spans [-500, 500] over the frame height and
// x keeps square pixels. Materials are the seven *_1K sets (PBRApp.cpp:1270-1463) assigned per 64x64
// pixel cell; F0 comes from the specular map (SPECULAR_TEXTURE permutation, Default.hlsl:91-92),
// metallic from the metalness map or g_Metallic = 0, and N from the normal map through
// NormalSampleToWorldSpace (LightingUtil.hlsl:203-214, not renormalised) with T = +x, B = -z, N = +y.
void fill_plane(const pbr_scene_desc& sc, int y, Row r) {
    const pbr_scene_assets* as = sc.assets;
    const int T = as->mat_size, M = as->num_materials;
    const float s = 1000.0f / (float)sc.height;
    for (int x = 0; x < sc.width; ++x) {
        r.p[kPosX][x] = ((float)x + 0.5f - 0.5f * (float)sc.width) * s;
        r.p[kPosY][x] = 0.0f;
        r.p[kPosZ][x] = (0.5f * (float)sc.height - ((float)y + 0.5f)) * s;
        const uint64_t cell = (uint64_t)(y / 64) * 65536u + (uint64_t)(x / 64);
        const int m = (int)(splitmix64(sc.seed ^ (cell * 0x9E3779B97F4A7C15ull)) % (uint64_t)M);
        const size_t t = ((size_t)m * T + (size_t)(y % T)) * T + (size_t)(x % T);
        const uint8_t* alb = as->mat_albedo + 3 * t;
        const uint8_t* spc = as->mat_specular + 3 * t;
        const uint8_t* nrm = as->mat_normal + 3 * t;
        r.p[kAr][x] = alb[0] / 255.0f;
        r.p[kAg][x] = alb[1] / 255.0f;
        r.p[kAb][x] = alb[2] / 255.0f;
        r.p[kF0r][x] = spc[0] / 255.0f;
        r.p[kF0g][x] = spc[1] / 255.0f;
        r.p[kF0b][x] = spc[2] / 255.0f;
        r.p[kRough][x] = as->mat_roughness[t] / 255.0f;
        r.p[kMetal][x] = as->mat_has_metallic[m] ? as->mat_metallic[t] / 255.0f : 0.0f;
        const float ntx = 2.0f * (nrm[0] / 255.0f) - 1.0f, nty = 2.0f * (nrm[1] / 255.0f) - 1.0f,
                    ntz = 2.0f * (nrm[2] / 255.0f) - 1.0f;
        // mul(normalT, float3x3(T, B, N)) = ntx*T + nty*B + ntz*N
        r.p[kNx][x] = ntx;
        r.p[kNy][x] = ntz;
        r.p[kNz][x] = -nty;
        r.p[kAo][x] = 1.0f;
    }
}

// ---- Kind 5: the reference scene -------------------------------------------------------------------
// 49 red spheres in a 7x7 grid (x = (i%7)*2.5 - 7.5, y = -(i/7)*2.5 - 2.5; roughness (i%7)/6, metallic
// 1 - (i/7)/6, albedo (1,0,0), F0 0.04; PBRApp.cpp:964-973, 1016-1022) and nine textured spheres on
// y = 0 (PBRApp.cpp:1023-1068), all SphereMesh radius 1 (PBRApp.cpp:515-560), ray-cast analytically
// from the camera instead of rasterised (the mesh's triangle interpolation is G-buffer content,
// parity-unpinned like the texture filtering). Per hit: PosW; NormalW = normalize(P - C) (Default.hlsl:50);
// SphereMesh's frame (Mesh.h:506-523): UV = (theta / 2pi, phi / pi), T = dP/dtheta = (-q.z, 0, q.x),
// B = cross(N, T) (neither normalised); materials per the reference's permutations (PBRApp.cpp:892-963,
// Default.hlsl:79-116); N = NormalSampleToWorldSpace (LightingUtil.hlsl:203-214, not renormalised);
// F0 resolved into the F0 plane (specular map, or lerp(0.04, albedo, metallic)).
struct RefSphere {
    float cx, cy;
    int tile;  // material tile (assets order: brick_modern, concrete_dirty, concrete_rough, grass_wild,
               // metal_bare, soil_mud, stone_wall), -1 = constant / special
    int kind;  // 0 red (index in `red`), 1 tiled, 2 rusted iron, 3 rock copper
    int red;
};

constexpr int kRefSpheres = 58;

RefSphere ref_sphere(int s) {
    if (s < 49) return RefSphere{(s % 7) * 2.5f - 3 * 2.5f, (s / 7) * -2.5f - 2.5f, -1, 0, s};
    static const RefSphere textured[9] = {
        {0.0f, 0.0f, -1, 2, 0},    // sphere_rust           (rusted_iron: metallic + roughness maps)
        {-2.5f, 0.0f, -1, 3, 0},   // sphere_rock_copper    (maps not among the committed tiles: constants)
        {-5.0f, 0.0f, 0, 1, 0},    // sphere_brick_modern
        {-7.5f, 0.0f, 1, 1, 0},    // sphere_concrete_dirty
        {-10.0f, 0.0f, 2, 1, 0},   // sphere_concrete_rough
        {2.5f, 0.0f, 3, 1, 0},     // sphere_grass_wild
        {5.0f, 0.0f, 4, 1, 0},     // sphere_metal_bare
        {7.5f, 0.0f, 5, 1, 0},     // sphere_soil_mud
        {10.0f, 0.0f, 6, 1, 0}};   // sphere_stone_wall
    return textured[s - 49];
}

struct Basis {
    double eye[3], f[3], r[3], u[3], t;
};

Basis camera_basis(const pbr_scene_desc& sc) {
    pbr_camera def = {{0.0f, 0.0f, -5.0f}, {0.0f, 0.0f, 0.0f}, (float)(M_PI / 4.0), 0.0f};
    const pbr_camera& c = sc.camera ? *sc.camera : def;
    Basis b;
    double f[3] = {(double)c.target[0] - c.eye[0], (double)c.target[1] - c.eye[1], (double)c.target[2] - c.eye[2]};
    double fl = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    for (int i = 0; i < 3; ++i) b.eye[i] = c.eye[i], b.f[i] = f[i] / fl;
    // left-handed: right = cross(up, forward), up' = cross(forward, right)
    double r[3] = {b.f[2], 0.0, -b.f[0]};
    double rl = std::sqrt(r[0] * r[0] + r[2] * r[2]);
    for (int i = 0; i < 3; ++i) b.r[i] = r[i] / rl;
    b.u[0] = b.f[1] * b.r[2] - b.f[2] * b.r[1];
    b.u[1] = b.f[2] * b.r[0] - b.f[0] * b.r[2];
    b.u[2] = b.f[0] * b.r[1] - b.f[1] * b.r[0];
    b.t = std::tan(0.5 * (double)c.fov_y);
    return b;
}

void fill_reference(const pbr_scene_desc& sc, int y, Row r) {
    const pbr_scene_assets* as = sc.assets;
    const Basis b = camera_basis(sc);
    const double aspect = (double)sc.width / (double)sc.height;
    const int T = as->mat_size, RS = as->rust_size;
    for (int x = 0; x < sc.width; ++x) {
        const double sx = (2.0 * (x + 0.5) / sc.width - 1.0) * b.t * aspect, sy = (1.0 - 2.0 * (y + 0.5) / sc.height) * b.t;
        double d[3];
        for (int i = 0; i < 3; ++i) d[i] = b.f[i] + sx * b.r[i] + sy * b.u[i];
        const double dl = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        for (int i = 0; i < 3; ++i) d[i] /= dl;
        // nearest hit within the camera's [near, far] = [0.1, 100] (BuildCamera, PBRApp.cpp:654)
        double best = 100.0;
        int hit = -1;
        for (int s = 0; s < kRefSpheres; ++s) {
            const RefSphere sp = ref_sphere(s);
            const double o[3] = {b.eye[0] - sp.cx, b.eye[1] - sp.cy, b.eye[2]};
            const double bb = o[0] * d[0] + o[1] * d[1] + o[2] * d[2];
            const double cc = o[0] * o[0] + o[1] * o[1] + o[2] * o[2] - 1.0;
            const double disc = bb * bb - cc;
            if (disc < 0.0) continue;
            const double sq = std::sqrt(disc);
            double tt = -bb - sq;
            if (tt < 0.1) tt = -bb + sq;  // eye inside / behind the near plane: the far side
            if (tt >= 0.1 && tt < best) best = tt, hit = s;
        }
        set_cov(r, x, hit >= 0);
        r.p[kAo][x] = 1.0f;
        if (hit < 0) {  // background: the view direction for the sky pass (Skybox.hlsl:24, 41)
            r.p[kPosX][x] = (float)(b.eye[0] + d[0] * 100.0);
            r.p[kPosY][x] = (float)(b.eye[1] + d[1] * 100.0);
            r.p[kPosZ][x] = (float)(b.eye[2] + d[2] * 100.0);
            r.p[kNx][x] = (float)d[0];
            r.p[kNy][x] = (float)d[1];
            r.p[kNz][x] = (float)d[2];
            r.p[kAr][x] = r.p[kAg][x] = r.p[kAb][x] = 0.0f;
            r.p[kMetal][x] = 0.0f;
            r.p[kRough][x] = 1.0f;
            r.p[kF0r][x] = r.p[kF0g][x] = r.p[kF0b][x] = 0.04f;
            continue;
        }
        const RefSphere sp = ref_sphere(hit);
        const double P[3] = {b.eye[0] + d[0] * best, b.eye[1] + d[1] * best, b.eye[2] + d[2] * best};
        const double q[3] = {P[0] - sp.cx, P[1] - sp.cy, P[2]};
        const double ql = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
        const float nw[3] = {(float)(q[0] / ql), (float)(q[1] / ql), (float)(q[2] / ql)};
        r.p[kPosX][x] = (float)P[0];
        r.p[kPosY][x] = (float)P[1];
        r.p[kPosZ][x] = (float)P[2];
        double theta = std::atan2(q[2], q[0]);
        if (theta < 0.0) theta += 2.0 * M_PI;
        const double uu = theta / (2.0 * M_PI), vv = std::acos(std::fmin(std::fmax(q[1] / ql, -1.0), 1.0)) / M_PI;
        const float tg[3] = {(float)-q[2], 0.0f, (float)q[0]};  // dP/dtheta
        const float bt[3] = {nw[1] * tg[2] - nw[2] * tg[1], nw[2] * tg[0] - nw[0] * tg[2], nw[0] * tg[1] - nw[1] * tg[0]};
        float alb[3], f0[3], metal, rough, n[3] = {nw[0], nw[1], nw[2]};
        bool has_spec = false;
        if (sp.kind == 0) {  // textureless red sphere (PBRApp.cpp:964-973)
            alb[0] = 1.0f, alb[1] = 0.0f, alb[2] = 0.0f;
            rough = (float)(sp.red % 7) / 6.0f;
            metal = 1.0f - (float)(sp.red / 7) / 6.0f;
        } else if (sp.kind == 2) {  // rusted iron: metallic + roughness maps (basecolor/normal absent, F6)
            const int tx = std::min(RS - 1, (int)(uu * RS)), ty = std::min(RS - 1, (int)(vv * RS));
            alb[0] = alb[1] = alb[2] = 0.5f;
            metal = (float)as->rust_metallic[(size_t)ty * RS + tx] / 255.0f;
            rough = (float)as->rust_roughness[(size_t)ty * RS + tx] / 255.0f;
        } else if (sp.kind == 3) {  // rock copper: constant copper-like values (maps not committed)
            alb[0] = 0.95f, alb[1] = 0.64f, alb[2] = 0.54f;
            metal = 1.0f;
            rough = 0.35f;
        } else {
            const int tx = std::min(T - 1, (int)(uu * T)), ty = std::min(T - 1, (int)(vv * T));
            const size_t t = ((size_t)sp.tile * T + (size_t)ty) * T + (size_t)tx;
            const uint8_t* a = as->mat_albedo + 3 * t;
            const uint8_t* sv = as->mat_specular + 3 * t;
            const uint8_t* nm = as->mat_normal + 3 * t;
            for (int c = 0; c < 3; ++c) alb[c] = a[c] / 255.0f, f0[c] = sv[c] / 255.0f;
            has_spec = true;
            rough = as->mat_roughness[t] / 255.0f;
            metal = as->mat_has_metallic[sp.tile] ? as->mat_metallic[t] / 255.0f : 0.0f;  // g_Metallic = 0
            const float nt[3] = {2.0f * (nm[0] / 255.0f) - 1.0f, 2.0f * (nm[1] / 255.0f) - 1.0f,
                                 2.0f * (nm[2] / 255.0f) - 1.0f};
            for (int c = 0; c < 3; ++c) n[c] = nt[0] * tg[c] + nt[1] * bt[c] + nt[2] * nw[c];  // mul(normalT, TBN)
        }
        if (!has_spec)
            for (int c = 0; c < 3; ++c) f0[c] = lerp_h(0.04f, alb[c], metal);  // Default.hlsl:94-95
        r.p[kNx][x] = n[0];
        r.p[kNy][x] = n[1];
        r.p[kNz][x] = n[2];
        r.p[kAr][x] = alb[0];
        r.p[kAg][x] = alb[1];
        r.p[kAb][x] = alb[2];
        r.p[kMetal][x] = metal;
        r.p[kRough][x] = rough;
        r.p[kF0r][x] = f0[0];
        r.p[kF0g][x] = f0[1];
        r.p[kF0b][x] = f0[2];
    }
}

bool assets_ok(const pbr_scene_desc* sc) {
    const pbr_scene_assets* as = sc->assets;
    if (!as) return false;
    if (sc->kind == PBR_SCENE_SPHERE_RUSTEDIRON || sc->kind == PBR_SCENE_RANDOM_COVERED)
        return as->rust_metallic && as->rust_roughness && as->rust_size > 0;
    if (sc->kind == PBR_SCENE_REFERENCE_SPHERES)
        return as->rust_metallic && as->rust_roughness && as->rust_size > 0 && as->mat_albedo && as->mat_specular &&
               as->mat_roughness && as->mat_metallic && as->mat_has_metallic && as->mat_normal &&
               as->num_materials >= 7 && as->mat_size > 0;
    if (sc->kind == PBR_SCENE_PLANE_MATERIALS)
        return as->mat_albedo && as->mat_specular && as->mat_roughness && as->mat_metallic && as->mat_has_metallic &&
               as->mat_normal && as->num_materials > 0 && as->mat_size > 0;
    return false;
}

}  // namespace

extern "C" int64_t pbr_gbuffer_fill(const pbr_scene_desc* scene, int32_t row_begin, int32_t row_end,
                                    float* const* planes, int64_t row_stride, int32_t n_threads) {
    return pbr_gbuffer_fill_coverage(scene, row_begin, row_end, planes, row_stride, nullptr, 0, n_threads);
}

extern "C" int64_t pbr_gbuffer_fill_coverage(const pbr_scene_desc* scene, int32_t row_begin, int32_t row_end,
                                             float* const* planes, int64_t row_stride, uint8_t* coverage,
                                             int64_t coverage_stride, int32_t n_threads) {
    if (coverage && scene && coverage_stride < scene->width) return PBR_ERR_INVALID_ARGUMENT;
    if (!scene || !planes || scene->width <= 0 || scene->height <= 0) return PBR_ERR_INVALID_ARGUMENT;
    if (row_begin < 0 || row_end < row_begin || row_end > scene->height || row_stride < scene->width)
        return PBR_ERR_INVALID_ARGUMENT;
    if (!assets_ok(scene)) return PBR_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < 15; ++i)
        if (!planes[i]) return PBR_ERR_INVALID_ARGUMENT;
    const int rows = row_end - row_begin;
    if (rows == 0) return 0;
    int nt = n_threads < 1 ? 1 : n_threads;
    if (nt > rows) nt = rows;
    if (nt > 256) nt = 256;
    std::vector<int64_t> covered(nt, 0);
    auto work = [&](int t) {
        const int r0 = row_begin + (int)((int64_t)rows * t / nt), r1 = row_begin + (int)((int64_t)rows * (t + 1) / nt);
        for (int y = r0; y < r1; ++y) {
            Row r;
            for (int i = 0; i < 15; ++i) r.p[i] = planes[i] + (int64_t)(y - row_begin) * row_stride;
            r.cov = coverage ? coverage + (int64_t)(y - row_begin) * coverage_stride : nullptr;
            switch (scene->kind) {
                case PBR_SCENE_SPHERE_RUSTEDIRON: covered[t] += fill_sphere(*scene, y, r); break;
                case PBR_SCENE_RANDOM_COVERED: fill_random_covered(*scene, y, r); covered[t] += scene->width; break;
                case PBR_SCENE_REFERENCE_SPHERES: {
                    Row rc = r;
                    std::vector<uint8_t> tmp;
                    if (!rc.cov) tmp.resize((size_t)scene->width), rc.cov = tmp.data();
                    fill_reference(*scene, y, rc);
                    for (int x = 0; x < scene->width; ++x) covered[t] += rc.cov[x];
                    break;
                }
                default: fill_plane(*scene, y, r); covered[t] += scene->width; break;
            }
            if (r.cov && scene->kind != PBR_SCENE_SPHERE_RUSTEDIRON && scene->kind != PBR_SCENE_REFERENCE_SPHERES)
                std::memset(r.cov, 1, (size_t)scene->width);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    int64_t total = 0;
    for (auto c : covered) total += c;
    return total;
}

extern "C" int pbr_scene_pass(const pbr_scene_desc* scene, int32_t n_lights, pbr_light* lights, pbr_pass_desc* pass) {
    if (!scene || !pass || n_lights < 0 || n_lights > PBR_MAX_LIGHTS || (n_lights > 0 && !lights))
        return PBR_ERR_INVALID_ARGUMENT;
    std::memset(pass, 0, sizeof(*pass));
    // PBRApp.cpp:478 ambient 0.03; Material.h:16-19 FresnelR0 0.04, opacity 1
    for (int i = 0; i < 3; ++i) {
        pass->ambient_light[i] = 0.03f;
        pass->fresnel_r0[i] = 0.04f;
    }
    pass->opacity = 1.0f;
    pass->eye_pos_w[0] = 0.0f;
    pass->eye_pos_w[1] = 0.0f;
    pass->eye_pos_w[2] = -5.0f;  // BuildCamera, PBRApp.cpp:652-659
    pass->ambient_mode = PBR_AMBIENT_CONSTANT;
    pass->num_point_lights = n_lights;
    pass->lights = lights;
    if (scene->kind == PBR_SCENE_REFERENCE_SPHERES) {  // PBRApp.cpp:480-487: four directional lights
        if (n_lights != 4) return PBR_ERR_INVALID_ARGUMENT;
        static const float dirs[4][3] = {{0.57735f, 0.57735f, 0.57735f}, {0.57735f, -0.57735f, 0.57735f},
                                         {-0.57735f, 0.57735f, 0.57735f}, {-0.57735f, -0.57735f, 0.57735f}};
        for (int i = 0; i < 4; ++i) {
            std::memset(&lights[i], 0, sizeof(pbr_light));
            lights[i].spot_power = 64.0f;
            for (int c = 0; c < 3; ++c) lights[i].strength[c] = 0.25f, lights[i].direction[c] = dirs[i][c];
        }
        pass->num_point_lights = 0;
        pass->num_dir_lights = 4;
        if (scene->camera)
            for (int c = 0; c < 3; ++c) pass->eye_pos_w[c] = scene->camera->eye[c];
        return PBR_OK;
    }
    const uint64_t ls = scene->seed ^ kLightStream;
    const float s = 1000.0f / (float)(scene->height > 0 ? scene->height : 1);
    const float half_w = 0.5f * (float)scene->width * s;
    for (int i = 0; i < n_lights; ++i) {
        pbr_light& L = lights[i];
        std::memset(&L, 0, sizeof(L));
        L.spot_power = 64.0f;  // d3dUtil.h:147 default
        L.direction[1] = -1.0f;
        if (scene->kind == PBR_SCENE_SPHERE_RUSTEDIRON) {
            // the commented-out point light 0 of PBRApp.cpp:490-491
            L.position[0] = 20.0f, L.position[1] = 20.0f, L.position[2] = -20.0f;
            L.strength[0] = L.strength[1] = L.strength[2] = 100.0f;
        } else if (scene->kind == PBR_SCENE_PLANE_MATERIALS) {
            L.position[0] = -half_w + 2.0f * half_w * u01(ls, (uint64_t)i, 0);
            L.position[1] = 5.0f + 15.0f * u01(ls, (uint64_t)i, 1);
            L.position[2] = -500.0f + 1000.0f * u01(ls, (uint64_t)i, 2);
            for (int c = 0; c < 3; ++c) L.strength[c] = 100.0f * u01(ls, (uint64_t)i, 3 + c);
        } else {
            L.position[0] = -20.0f + 40.0f * u01(ls, (uint64_t)i, 0);
            L.position[1] = -20.0f + 40.0f * u01(ls, (uint64_t)i, 1);
            L.position[2] = -20.0f + 20.0f * u01(ls, (uint64_t)i, 2);
            for (int c = 0; c < 3; ++c) L.strength[c] = 100.0f * u01(ls, (uint64_t)i, 3 + c);
        }
    }
    if (scene->kind == PBR_SCENE_PLANE_MATERIALS) {
        pass->eye_pos_w[0] = 0.0f;
        pass->eye_pos_w[1] = 800.0f;
        pass->eye_pos_w[2] = 0.0f;
        pass->flags = PBR_FLAG_F0_PLANE;
    }
    return PBR_OK;
}

// This unit's build record (pbr_build_info.h, pbr_build_info).
#include "pbr_build_info.h"
extern "C" __attribute__((used, visibility("default"))) const char pbr_unit_info_gbuffer_fill[] =
    PBR_UNIT_INFO("gbuffer_fill", "");
