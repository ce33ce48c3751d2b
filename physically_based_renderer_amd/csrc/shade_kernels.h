// shade_kernels.h -- internal launch interface between the C-ABI layer and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "pbr_census.h"

namespace pbr {

constexpr int kAmbientConstant = 0;
constexpr int kAmbientIblDiffuse = 1;

// The 15 SoA planes in pbr_gbuffer_soa order: pos xyz, normal xyz, albedo rgb, metallic,
// roughness, ao, f0 rgb, then [15] the opacity plane (PBR_FLAG_ALPHA_TEST). Unused planes may alias plane 0
// (they are never read).
struct GBufferArgs {
    const float* plane[16];
    int width, height;
    int64_t row_stride;
    bool pairs_aligned;  // every read plane 8-byte aligned and row_stride even: 8-byte pair loads
    bool alpha_test;     // PBR_FLAG_ALPHA_TEST: clip on plane[15] (Default.hlsl:111-113)
};

// Pass constants passed by value as kernel arguments (the shading subset of cbPass / cbMaterial).
struct PassArgs {
    float eye[3];
    float ambient[3];
    float fresnel_r0[3];
    float opacity;
    int n_dir, n_point, n_spot;
    int env_w, env_h;
    int sky_w, sky_h;
    int eye_ok;  // the eye position is inside the fast-path window (0 or |x| in [2^-20, 2^20]), host-checked
    int balanced;  // untiled pass whose point lights take the wave-balanced lists (pbr_balanced.h): 0 no,
                   // 1 faithful pass (no spot lights), 2 exact pass (no spot or directional lights)
    int faithful;  // PBR_FLAG_FAITHFUL: 0 off; 1 on (host preconditions hold); 2 on, culled pass with > 64
                   // lights: the kernel counts each wave's summed terms against the bound's 64
};

constexpr int kOutRgba32f = 0;
constexpr int kOutRgba8 = 1;

// Where and how a pass writes its pixels (pbr_frame_desc).
struct FrameArgs {
    void* out;                 // float4 (kOutRgba32f) or uint32 RGBA8 (kOutRgba8) per pixel
    int64_t out_stride;        // pixels
    int format;
    const uint8_t* coverage;   // nullptr = every pixel is geometry; else 0 = background (sky pass)
    int64_t coverage_stride;   // bytes
    const float4* sky;         // sky_w * sky_h RGBA fp32 (required when coverage != nullptr)
    int width, height;         // the frame (= the G-buffer's; PBR_DEBUG_BOUNDS builds check stores against it)
};

// One statistics record (int32 each): its fields, summed over the pass by pbr_last_pass_stats.
enum StatField {
    kStatCullKept = 0,        // culled passes: surviving point/spot lights of the culling unit
    kStatCullTiles = 1,       // culled passes: 1 when the culling unit has geometry
    kStatExactPixels = 2,     // geometry pixels whose light sum the exact path redid
    kStatLightTerms = 3,      // (geometry pixel, light) terms the light loops evaluated
    kStatGeometryPixels = 4,  // geometry pixels
    kStatBackfaceTests = 5,   // balanced passes: (pixel, point light) back-face tests of pass 1
    kStatsPerBlock = 6
};
constexpr int kBalMaxLights = 64;  // point lights per wave-balanced pass (one 64-bit live mask per pixel)

struct LaunchArgs {
    GBufferArgs gb;
    PassArgs ps;
    const float4* lights;  // 3 float4 per light (the reference's 48-byte Light)
    const float4* env;     // env_w * env_h RGBA fp32, or nullptr
    FrameArgs frame;
    // kStatsPerBlock ints per statistics slot (shade_stat_slots_per_tile slots per workgroup, workgroup =
    // blockIdx.y * gridDim.x + blockIdx.x): surviving point/spot lights summed over its culling units and the
    // number of culling units with geometry (both 0 without CULL; the pair layout culls per wave = 64x2
    // pixels and keeps one slot per wave, the one-pixel layout culls per workgroup = 32x8), and the geometry
    // pixels the exact path redid. Plain stores: one same-address global atomic per tile serialised the
    // whole grid (0.29 ms per 4K frame). May be nullptr.
    int32_t* tile_kept;
    int ambient_mode;
    bool f0_plane, apply_ao, cull;
    bool exact_only;  // PBR_FLAG_EXACT_ONLY: skip the exact fast path (validation mode)
    int pixels_per_thread;  // 1 (32x8 tiles) or 2 (64x8 tiles, packed pairs)
    // Shade with the lean pair kernel (uniform-loop passes without a sky pass or EXACT_ONLY, pixels_per_thread 2;
    // tile_kept required): shade_lean_kernel.
    bool lean;
};

hipError_t launch_shade(const LaunchArgs& a, hipStream_t stream);
// The kernel launch_shade launches for `a`, as rocprofv3 names it without the argument list.
std::string launched_kernel(const LaunchArgs& a);
// Number of tiles (workgroups) launch_shade uses for a width x height G-buffer.
int64_t shade_tile_count(int width, int height, int pixels_per_thread);
// Statistics records per tile: one per wave in the pair layout, one per workgroup in the one-pixel layout.
int shade_stat_slots_per_tile(int pixels_per_thread);
hipError_t debug_bal_profile(unsigned long long* out8, bool reset);  // PBR_BAL_PROFILE builds only
hipError_t debug_wave_timeline(unsigned long long* buf, long long cap);  // PBR_WAVE_TIMELINE builds only
hipError_t debug_bounds_publish(uint32_t* buf);  // PBR_DEBUG_BOUNDS builds only (pbr_debug_bounds.h)
hipError_t launch_decode_unorm16(const uint16_t* src, float4* dst, int n_texels, hipStream_t stream);

}  // namespace pbr
