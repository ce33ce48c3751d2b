/*
 * oracle/pbr_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's per-pixel shading path:
 *   PS                 /root/reference/Source/Shaders/Default.hlsl:47-161
 *   ComputeLighting &  /root/reference/Source/Shaders/LightingUtil.hlsl:35-225
 *   cbuffer layouts    /root/reference/Source/Shaders/Core.hlsl:35-81
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * Parity is pinned: tests/golden/ holds vectors produced by oracle/_ref (the reference's own
 * pixel-shader text -- Default.hlsl's PS with Core.hlsl and LightingUtil.hlsl, Skybox.hlsl's PS -- compiled
 * as C++), and tests/test_oracle_golden.py checks this file against them.
 *
 * The oracle has its own flat interface (no product header), so a product bug in struct
 * marshalling cannot hide behind a shared definition.
 */
#ifndef PBR_ORACLE_H
#define PBR_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One light, exactly the reference cbuffer element (LightingUtil.hlsl:9-17, d3dUtil.h:144-152): 48 B. */
typedef struct oracle_light {
    float strength[3];
    float spot_power;
    float direction[3];
    float pad0;
    float position[3];
    float pad1;
} oracle_light;

enum { ORACLE_AMBIENT_CONSTANT = 0, ORACLE_AMBIENT_IBL_DIFFUSE = 1 };

/* Plane order of the structure-of-arrays G-buffer. */
enum {
    ORACLE_PX = 0, ORACLE_PY, ORACLE_PZ,
    ORACLE_NX, ORACLE_NY, ORACLE_NZ,
    ORACLE_AR, ORACLE_AG, ORACLE_AB,
    ORACLE_METAL, ORACLE_ROUGH, ORACLE_AO,
    ORACLE_F0R, ORACLE_F0G, ORACLE_F0B,
    ORACLE_OPACITY,        /* the ALPHA_TEST permutation's opacity map (Default.hlsl:111-112) */
    ORACLE_NUM_PLANES
};

typedef struct oracle_pass {
    float eye[3];          /* cbPass g_CameraPosW          Core.hlsl:43 */
    float ambient[3];      /* cbPass g_AmbientLight.rgb    Core.hlsl:51 */
    float fresnel_r0[3];   /* cbMaterial g_FresnelR0       Core.hlsl:68 */
    float opacity;         /* cbMaterial g_Opacity         Core.hlsl:74 */
    int32_t n_dir, n_point, n_spot;   /* NUM_*_LIGHTS      Core.hlsl:1-12 */
    int32_t ambient_mode;  /* ORACLE_AMBIENT_*  */
    int32_t use_f0_plane;  /* SPECULAR_TEXTURE permutation  Default.hlsl:91-96 */
    int32_t apply_ao;      /* extension: ambient *= AO (reference: off) */
    int32_t alpha_test;    /* ALPHA_TEST permutation (PBRApp.cpp:750-765): fragOpacity = the opacity plane,
                              clip(fragOpacity - 0.1f) leaves the pixel's output untouched  Default.hlsl:111-113 */
} oracle_pass;

/*
 * Shade rows [0, height) of a width x height SoA G-buffer.
 *   planes[ORACLE_NUM_PLANES]  host fp32 planes; AO / F0 planes may be NULL when unused
 *   stride                     elements between rows of a plane
 *   lights                     n_dir + n_point + n_spot lights, in that order
 *   env_rgba16                 env_w * env_h * 4 u16 texels (IBL mode only; else NULL)
 *   out                        RGBA fp32, out_stride pixels between rows
 *   n_threads                  >= 1 (row-partitioned pthreads)
 * Returns 0 on success, negative on bad arguments.
 */
int oracle_shade(int width, int height, int64_t stride, const float* const* planes,
                 const oracle_pass* pass, const oracle_light* lights,
                 const uint16_t* env_rgba16, int env_w, int env_h,
                 float* out, int64_t out_stride, int n_threads);

/* ---- Frame composition (product: pbr_shade_frame) --------------------------------------------- */

enum { ORACLE_OUTPUT_RGBA32F = 0, ORACLE_OUTPUT_RGBA8 = 1 };

typedef struct oracle_frame {
    const float* env_rgba;    /* IBL texture as RGBA fp32 (decode UNORM16 with oracle_decode_unorm16) */
    int32_t env_w, env_h;
    const float* sky_rgba;    /* sky texture g_SkyArray[0] (Skybox.hlsl:45), RGBA fp32 */
    int32_t sky_w, sky_h;
    const uint8_t* coverage;  /* NULL = all geometry; else 0 = background -> Skybox.hlsl PS */
    int64_t coverage_stride;  /* bytes */
    int32_t format;           /* ORACLE_OUTPUT_*: RGBA fp32 (16 B/px) or RGBA8 UNORM (4 B/px) */
    int32_t pad0;
} oracle_frame;

/* As oracle_shade, with the sky pass on background pixels and the output format of `frame`. */
int oracle_shade_frame(int width, int height, int64_t stride, const float* const* planes,
                       const oracle_pass* pass, const oracle_light* lights, const oracle_frame* frame,
                       void* out, int64_t out_stride, int n_threads);

/* R16G16B16A16_UNORM decode: dst[i] = (float)src[i] / 65535.0f. */
void oracle_decode_unorm16(const uint16_t* src, int64_t n_values, float* dst);

/* D3D FLOAT -> UNORM8: NaN -> 0, clamp [0, 1], c * 255 + 0.5 (fp32), truncate. */
uint8_t oracle_unorm8(float c);

#ifdef __cplusplus
}
#endif
#endif
