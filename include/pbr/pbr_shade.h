/*
 * pbr_shade.h -- C ABI of the MI355X (gfx950) G-buffer shading library, libpbrshade.so.
 *
 * Drop-in for the hot path of trevordblack/Physically_Based_Renderer: the per-pixel Cook-Torrance
 * pixel shader PS (Source/Shaders/Default.hlsl:47-161) and everything it calls in
 * Source/Shaders/LightingUtil.hlsl:35-225, which the reference runs by DrawIndexedInstanced
 * (Source/App/PBRApp.cpp:1133) inside PBRApp::Draw (PBRApp.cpp:245-352). The D3D12 rasteriser
 * front-end is replaced by a flat structure-of-arrays G-buffer the caller fills (pbr_gbuffer_fill
 * below does it on the host for the benchmark scenes).
 *
 * Conventions (mirroring the reference's HRESULT/ThrowIfFailed checking, d3dUtil.h:156-163):
 *   - every function returns int: 0 = PBR_OK, negative = pbr_status; no exception crosses the ABI;
 *   - the caller owns every buffer passed in; the library never frees them;
 *   - device work is stream-ordered and asynchronous on the hipStream_t given (NULL = default
 *     stream); a context is bound to one device and is reentrant across streams, like the
 *     reference's 3-deep frame-resource ring (FrameResource.h:111-140, PBRApp.cpp:220-243): every
 *     pbr_set_pass uploads into its own device light slot, a pass reads the slot of the
 *     pbr_set_pass before it and waits (stream-side) for that upload when it was made on another
 *     stream, and a slot or texture is overwritten only after the queued passes that read it, on
 *     whatever stream they run. Host calls on one context are serialised by its mutex; the host
 *     order of pbr_set_pass and pbr_shade_* calls decides which pass a shade uses. Contexts expect a
 *     small, long-lived set of streams: the first call on a new stream synchronises the device once,
 *     and past 16 streams the context forgets all but its last one then. Let a stream's passes
 *     finish before destroying it (a new stream may reuse its handle value). A light slot or
 *     texture that grows (more lights than the slot held, a larger map) is released and
 *     reallocated in stream order on the calling stream (hipFreeAsync / hipMallocAsync after
 *     stream-side waits for its readers): no device synchronisation. pbr_set_env_map and
 *     pbr_set_sky_map synchronise their own stream (the host texels may be released on return),
 *     and pbr_set_pass may wait on the host for the upload that last used its staging slot: call
 *     them outside a graph capture. pbr_shade_* on a stream the context already knows queues only
 *     stream-ordered work (event records and waits, the kernel).
 * Plain C types only (hipStream_t is passed as void*).
 */
#ifndef PBR_SHADE_H
#define PBR_SHADE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBR_ABI_VERSION 9
#define PBR_MAX_LIGHTS 4096 /* the reference's cbuffer holds MAX_LIGHTS = 16 (LightingUtil.hlsl:7) */

typedef enum pbr_status {
    PBR_OK = 0,
    PBR_ERR_INVALID_ARGUMENT = -1,
    PBR_ERR_NO_DEVICE = -2,
    PBR_ERR_OUT_OF_MEMORY = -3,
    PBR_ERR_LAUNCH = -4,
    PBR_ERR_HIP = -5,
    PBR_ERR_NOT_READY = -6, /* shade called before pbr_set_pass / IBL without pbr_set_env_map */
    PBR_ERR_UNSUPPORTED = -7
} pbr_status;

/* One light, byte-identical to the reference cbuffer element `Light` (LightingUtil.hlsl:9-17,
 * C++ mirror d3dUtil.h:144-152): 48 bytes, float4-aligned. Lights of a pass are ordered
 * directional [0, n_dir), point [n_dir, n_dir+n_point), spot [.., +n_spot) as ComputeLighting
 * expects (LightingUtil.hlsl:176-199). */
typedef struct pbr_light {
    float strength[3];
    float spot_power;   /* spot only */
    float direction[3]; /* directional / spot only */
    float pad0;
    float position[3];  /* point / spot only */
    float pad1;
} pbr_light;

typedef enum pbr_ambient_mode {
    PBR_AMBIENT_CONSTANT = 0,   /* g_AmbientLight * albedo: the active reference code, Default.hlsl:150 */
    PBR_AMBIENT_IBL_DIFFUSE = 1 /* the diffuse-IBL block of Default.hlsl:140-149 (commented out there) */
} pbr_ambient_mode;

enum pbr_pass_flags {
    PBR_FLAG_F0_PLANE = 1u << 0,    /* F0 from the G-buffer (SPECULAR_TEXTURE permutation, Default.hlsl:91-92);
                                       otherwise F0 = lerp(fresnel_r0, albedo, metallic) (Default.hlsl:94-95) */
    PBR_FLAG_APPLY_AO = 1u << 1,    /* extension: ambient *= AO. The reference never reads its AO slot. */
    PBR_FLAG_TILED_CULLING = 1u << 2, /* per-tile range culling of point/spot lights; output is
                                         bit-identical to the unculled pass ("exact culling") */
    PBR_FLAG_EXACT_ONLY = 1u << 3,    /* validation mode: never take the exact fast division/sqrt path
                                         ("exact fast path"); output is bit-identical, slower */
    PBR_FLAG_FAITHFUL = 1u << 4,      /* tolerance mode (ABI 4): the well-conditioned divisions of the BRDF
                                         (NDF, Smith G1(N.L), specular denominator, diffuse / PI,
                                         attenuation) use the hardware reciprocal (<= 1 ulp) instead of
                                         correct rounding; the ill-conditioned GGX chain and Fresnel stay
                                         exact. Output within 1e-5 relative of the reference evaluation
                                         (the north-star bar; bound 6.1e-6, tiled and wave-balanced passes
                                         6.4e-6; measured 6.3e-7), not bit-identical.
                                         Applies where every light term is >= 0 and the sum is short:
                                         <= 64 lights (with PBR_FLAG_TILED_CULLING: <= 64 surviving lights,
                                         counted per wave), non-negative strengths, ambient and env texels
                                         (checked on the host), albedo >= 0 and F0 in [0, 1] (checked per
                                         wave); elsewhere the pass stays exact. */
    PBR_FLAG_ALPHA_TEST = 1u << 5     /* ABI 6: the ALPHA_TEST permutation (alphaTestedPS, PBRApp.cpp:750-765,
                                         Default.hlsl:111-113): fragOpacity = the G-buffer's opacity plane;
                                         a pixel with fragOpacity - 0.1f < 0 is discarded (its output is left
                                         untouched), others get alpha = fragOpacity. Sky pixels are not tested. */
};

/* Per-frame constants: the shading subset of cbPass (Core.hlsl:35-61, FrameResource.h:19-44) and
 * cbMaterial (Core.hlsl:64-81, Material.h:10-29). */
typedef struct pbr_pass_desc {
    float eye_pos_w[3];     /* g_CameraPosW */
    float ambient_light[3]; /* g_AmbientLight.rgb */
    float fresnel_r0[3];    /* g_FresnelR0 (default 0.04) */
    float opacity;          /* g_Opacity -> output alpha (default 1) */
    int32_t num_dir_lights;   /* NUM_DIR_LIGHTS   (Core.hlsl:1-3)  */
    int32_t num_point_lights; /* NUM_POINT_LIGHTS (Core.hlsl:5-7)  */
    int32_t num_spot_lights;  /* NUM_SPOT_LIGHTS  (Core.hlsl:9-11) */
    int32_t ambient_mode;     /* pbr_ambient_mode */
    uint32_t flags;           /* pbr_pass_flags */
    const pbr_light* lights;  /* HOST pointer, num_dir+num_point+num_spot lights */
} pbr_pass_desc;

/* Structure-of-arrays G-buffer in DEVICE memory: one fp32 plane per channel, `row_stride`
 * elements between rows. Replaces the interpolated VertexOut + texture fetches of PS
 * (Default.hlsl:12-20, 79-116): N is the final (normal-mapped) normal, F0 optional. */
typedef struct pbr_gbuffer_soa {
    const float* pos_w[3];    /* PosW x, y, z */
    const float* normal_w[3]; /* N x, y, z */
    const float* albedo[3];   /* diffuseAlbedo r, g, b */
    const float* metallic;
    const float* roughness;
    const float* ao;          /* read only with PBR_FLAG_APPLY_AO; may be NULL otherwise */
    const float* f0[3];       /* read only with PBR_FLAG_F0_PLANE; may be NULL otherwise */
    int32_t width;
    int32_t height;
    int64_t row_stride;       /* elements; >= width */
    const float* opacity;     /* ABI 6: read only with PBR_FLAG_ALPHA_TEST (the opacity map, Default.hlsl:112);
                                 may be NULL otherwise */
} pbr_gbuffer_soa;

typedef struct pbr_context pbr_context;

/* Replaces device creation + root signature / PSO build (d3dApp.cpp:437-501, PBRApp.cpp:607-650,
 * 776-881). `device` is a HIP device ordinal. */
int pbr_context_create(int device, pbr_context** out_ctx);
int pbr_context_destroy(pbr_context* ctx);

/* Replaces UpdateMainPassCB + UploadBuffer::CopyData (PBRApp.cpp:455-502, UploadBuffer.h:53):
 * uploads the light list and constants, stream-ordered; `pass` may be reused on return. */
int pbr_set_pass(pbr_context* ctx, const pbr_pass_desc* pass, void* stream);

/* Replaces loading + binding the environment SRV (PBRApp.cpp:1205-1210, t0-t1): an R16G16B16A16_UNORM
 * texture, `texels` = HOST pointer to width*height*4 u16, row-major. Sampled with linear-wrap
 * filtering (g_SamLinearWrap, PBRApp.cpp:1157-1162) by the IBL_DIFFUSE ambient. */
int pbr_set_env_map(pbr_context* ctx, const uint16_t* texels, int32_t width, int32_t height, void* stream);

/* Replaces DrawIndexedInstanced(PS) (PBRApp.cpp:1133, Default.hlsl:47-161): shades every pixel of
 * `gb` with the current pass into `out_rgba` (DEVICE, fp32 RGBA, out_row_stride PIXELS between rows).
 * Asynchronous on `stream`. Pixels are independent, so a caller can shade a row band by offsetting
 * the plane pointers (multi-GPU row tiles). */
int pbr_shade_gbuffer(pbr_context* ctx, const pbr_gbuffer_soa* gb, float* out_rgba, int64_t out_row_stride,
                      void* stream);

/* ---- Frame composition: sky pass, output format, HDR textures (ABI 2) -------------------------- */

/* Output pixel formats. RGBA32F is what pbr_shade_gbuffer writes. RGBA8_UNORM is the reference's
 * back buffer (DXGI_FORMAT_R8G8B8A8_UNORM, d3dApp.h:124; presented by PBRApp::Draw, PBRApp.cpp:274-279),
 * converted with the D3D FLOAT -> UNORM rule: NaN -> 0, clamp to [0, 1], c * 255 + 0.5, truncate. */
typedef enum pbr_output_format {
    PBR_OUTPUT_RGBA32F = 0,
    PBR_OUTPUT_RGBA8_UNORM = 1
} pbr_output_format;

typedef struct pbr_frame_desc {
    void* out;                   /* DEVICE: RGBA32F 16 B/px (16-byte aligned) or RGBA8 4 B/px (4-byte aligned) */
    int64_t out_row_stride;      /* pixels between output rows, >= width */
    int32_t format;              /* pbr_output_format */
    int32_t pad0;
    /* Optional DEVICE coverage plane, one byte per pixel, `coverage_row_stride` bytes per row:
     * nonzero = geometry (shaded by PS, Default.hlsl:47-161); 0 = background, which gets the sky pass
     * of Skybox.hlsl:37-49 instead (the reference draws the sky dome where no geometry wrote depth,
     * PBRApp.cpp:319-320, 856-875). For a background pixel the G-buffer normal planes hold the sky
     * sample direction (the sky dome's interpolated local position, Skybox.hlsl:24); its other planes
     * are not used. NULL = every pixel is geometry. */
    const uint8_t* coverage;
    int64_t coverage_row_stride;
} pbr_frame_desc;

/* The sky texture g_SkyArray[0] (PBRApp.cpp:1200-1204, sampled by Skybox.hlsl:45 with g_SamLinearWrap):
 * R16G16B16A16_UNORM, HOST texels as pbr_set_env_map. Required when a frame has background pixels. */
int pbr_set_sky_map(pbr_context* ctx, const uint16_t* texels, int32_t width, int32_t height, void* stream);

/* fp32 RGBA variants of pbr_set_env_map / pbr_set_sky_map (HOST width*height*4 floats, e.g. a decoded
 * RGBE .hdr environment, Assets/<set>/<set>_Env.hdr): the texels are used as given, no UNORM decode. */
int pbr_set_env_map_f32(pbr_context* ctx, const float* texels, int32_t width, int32_t height, void* stream);
int pbr_set_sky_map_f32(pbr_context* ctx, const float* texels, int32_t width, int32_t height, void* stream);

/* pbr_shade_gbuffer with the frame options above, in one pass over the G-buffer (the sky and the
 * format conversion are fused into the shading kernel). Asynchronous on `stream`. */
int pbr_shade_frame(pbr_context* ctx, const pbr_gbuffer_soa* gb, const pbr_frame_desc* frame, void* stream);

/* Tiled-culling statistics of the last pass on `stream` (synchronises that stream; see
 * pbr_last_pass_stats for which pass), zeros when that pass did not cull:
 * total surviving point/spot lights summed over the culling tiles that hold geometry, and the number
 * of those tiles. A culling tile is one wave64's pixels (64x2 in the default pixel-pair layout, 32x8
 * workgroups in the one-pixel layout). The kernel writes per-workgroup counts (no atomics); this
 * call sums them on the host. */
int pbr_last_cull_stats(pbr_context* ctx, int64_t* sum_tile_lights, int64_t* num_tiles, void* stream);

/* Statistics of the last shading pass of the context (new; the reference has no counterpart). */
typedef struct pbr_pass_stats {
    int64_t workgroups;       /* workgroups of the pass (64x8-pixel tiles; 32x8 in the one-pixel layout) */
    int64_t culled;           /* 1 when the pass ran tiled culling, else 0 */
    int64_t cull_tiles;       /* culling tiles with geometry (0 without culling) */
    int64_t cull_tile_lights; /* surviving point/spot lights summed over those tiles (0 without culling) */
    int64_t exact_pixels;     /* geometry pixels whose light sum the exact path re-evaluated (inputs or
                                 intermediates outside the fast-path window; every geometry pixel with
                                 PBR_FLAG_EXACT_ONLY) */
    /* ABI 5: the work the light loops executed (what a FLOP count of the pass may credit). */
    int64_t light_terms;      /* (geometry pixel, light) terms evaluated: every light of the pass in the
                                 uniform loop, the survivors of the culling tile under PBR_FLAG_TILED_CULLING,
                                 the live (front-facing, in the wave-balanced lists) point lights plus the
                                 directional ones in a wave-balanced pass. The exact re-pass of
                                 exact_pixels is not counted. */
    int64_t geometry_pixels;  /* pixels shaded by PS (the coverage plane's non-zero pixels; all without one) */
    int64_t backface_tests;   /* wave-balanced passes: (pixel, point light) back-face tests of the list
                                 build (4 FMAs each); 0 otherwise */
} pbr_pass_stats;

/* Fill *out with the statistics of the last pbr_shade_gbuffer / pbr_shade_frame call on `stream`
 * (synchronises `stream`). Each stream keeps its own record, so passes on other streams never mix
 * into it; if the context has not shaded on `stream`, the context's last pass on any stream is
 * reported, and `stream` must then be ordered after that pass. All zero before the first pass.
 * The kernel writes one record per wave (workgroup in the one-pixel layout); this call sums them. */
int pbr_last_pass_stats(pbr_context* ctx, pbr_pass_stats* out, void* stream);

/* ABI 7: the kernel the last pass on `stream` launched (the same fallback as pbr_last_pass_stats), as the
 * profiler names it without its argument list, e.g. "shade_tile_kernel<1, false, false, false, 1>"
 * (the wave-balanced faithful lists) or "shade_lean_kernel<0, true, false, true, true>"; "" before the first
 * pass. The string is owned by the context and stays valid until the next pass on that stream. */
const char* pbr_last_pass_kernel(pbr_context* ctx, void* stream);

/* ABI 8: the bounds-checked kernel build (PBR_DEBUG_BOUNDS=1: `make -C physically_based_renderer_amd/csrc
 * debug-bounds`: physically_based_renderer_amd/_lib/debug_bounds/libpbrshade.so), the analogue of the reference's D3D12 debug layer
 * (d3dApp.cpp:443-444). Its kernels check every G-buffer, output, coverage, texel and light index (and the
 * wave-balanced lists' LDS indices) against the launch's extents; a violation is recorded, not trapped, and the
 * access is redirected to index 0. Synchronises the context's device, then copies its flags into `flags`
 * (16 words, may be NULL): flags[c] != 0 when index class c was violated (0 G-buffer, 1 output, 2 coverage,
 * 3 texel, 4 light, 5 LDS list), flags[8 + c] the last offending index; `reset` != 0 clears them. Every pass since
 * the first context on the device (or the last reset) counts. PBR_ERR_UNSUPPORTED from a product build. */
int pbr_debug_bounds(pbr_context* ctx, uint32_t* flags, int reset);

/* ---- Host G-buffer fill (replaces the VS + rasteriser front-end, Default.hlsl:22-45) ---------- */

typedef enum pbr_scene_kind {
    PBR_SCENE_SPHERE_RUSTEDIRON = 1, /* BASELINE config 1: ray-cast unit sphere, rustediron metal/rough */
    PBR_SCENE_RANDOM_COVERED = 2,    /* configs 2, 3, 5: fully covered synthetic G-buffer */
    PBR_SCENE_PLANE_MATERIALS = 4,   /* config 4: plane y = 0 seen top-down, seven *_1K material sets */
    PBR_SCENE_REFERENCE_SPHERES = 5  /* the reference's own scene: 49 red spheres + 9 textured spheres
                                        (PBRApp.cpp:964-973, 1016-1068) under its 4 directional lights */
} pbr_scene_kind;

/* A left-handed look-at camera with world up (0, 1, 0), like Camera (Camera.cpp:104-112). */
typedef struct pbr_camera {
    float eye[3];
    float target[3];
    float fov_y; /* radians */
    float pad0;
} pbr_camera;

/* Host-side texture tiles the scenes sample (owned by the caller). */
typedef struct pbr_scene_assets {
    const uint8_t* rust_metallic;  /* rust_size^2 u8 gray */
    const uint8_t* rust_roughness; /* rust_size^2 u8 gray */
    int32_t rust_size;
    const uint8_t* mat_albedo;     /* [num_materials][mat_size][mat_size][3] */
    const uint8_t* mat_specular;   /* [num_materials][mat_size][mat_size][3] */
    const uint8_t* mat_roughness;  /* [num_materials][mat_size][mat_size]    */
    const uint8_t* mat_metallic;   /* [num_materials][mat_size][mat_size]    */
    const uint8_t* mat_has_metallic; /* [num_materials] */
    const uint8_t* mat_normal;     /* [num_materials][mat_size][mat_size][3] */
    int32_t num_materials;
    int32_t mat_size;
} pbr_scene_assets;

typedef struct pbr_scene_desc {
    int32_t kind;         /* pbr_scene_kind */
    int32_t width;        /* full-frame size: pixel values depend on the global (x, y) only, */
    int32_t height;       /* never on how rows are partitioned across calls or ranks */
    uint64_t seed;
    const pbr_scene_assets* assets;
    const pbr_camera* camera; /* kind 5 only; NULL = the reference's initial camera: eye (0, 0, -5) looking
                                 down +z, fovY pi/4 (BuildCamera, PBRApp.cpp:652-659) */
} pbr_scene_desc;

/* Fills rows [row_begin, row_end) of the full frame into HOST planes laid out like
 * pbr_gbuffer_soa (15 planes in the order pos xyz, normal xyz, albedo rgb, metallic, roughness,
 * ao, f0 rgb; `planes[i]` points at row `row_begin`; `row_stride` elements). Returns the number of
 * covered (non-background) pixels, or a negative pbr_status. */
int64_t pbr_gbuffer_fill(const pbr_scene_desc* scene, int32_t row_begin, int32_t row_end, float* const* planes,
                         int64_t row_stride, int32_t n_threads);

/* pbr_gbuffer_fill that also writes the coverage plane pbr_shade_frame consumes: one byte per pixel,
 * 1 = geometry, 0 = background (config 1's sky around the sphere; the other scenes are fully covered).
 * Background pixels get the view direction in their normal planes (the sky dome point they see). */
int64_t pbr_gbuffer_fill_coverage(const pbr_scene_desc* scene, int32_t row_begin, int32_t row_end,
                                  float* const* planes, int64_t row_stride, uint8_t* coverage,
                                  int64_t coverage_stride, int32_t n_threads);

/* The light list and pass constants of a benchmark scene (`n_lights` point lights; kind 1 uses one
 * light at (20, 20, -20), strength 100, PBRApp.cpp:490-491; kind 5 uses the reference's four
 * directional lights, PBRApp.cpp:480-487, and needs n_lights == 4). `pass->lights` is set to `lights`. */
int pbr_scene_pass(const pbr_scene_desc* scene, int32_t n_lights, pbr_light* lights, pbr_pass_desc* pass);

const char* pbr_strerror(int status);
/* Last HIP error string recorded by the context (empty if none). */
const char* pbr_last_error(const pbr_context* ctx);
int pbr_abi_version(void);
/* ABI 9: what the library was built from, as JSON: {"abi": 9, "units": [{"unit", "sources_sha", "flavor", "cflags",
 * "switches": {...}}, ...]} -- one record per compilation unit (pbr_context, shade_kernels, shade_kernels_bal,
 * gbuffer_fill): the stamp of the sources it was compiled from (sha256 of the csrc sources, the Makefile and this header, first
 * 16 hex digits), the build flavor ("product" for the Makefile's default target without EXTRA flags; "debug_bounds",
 * "asan", "custom: ...", "variant: ..." otherwise), its extra compiler flags and every build switch's value. A program
 * that quotes a measurement can check it ran the product build of a given checkout. Static storage. */
const char* pbr_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* PBR_SHADE_H */
