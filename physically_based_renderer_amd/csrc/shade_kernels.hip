// shade_kernels.hip -- gfx950 kernels for the G-buffer shading hot path.
//
// One workgroup = one 32x8-pixel screen tile = 256 work-items = 4 wave64s; wave w owns tile rows
// 2w and 2w+1, so every per-plane load is two fully used 128-byte row segments and every RGBA
// store is two 512-byte segments. The light list is staged through LDS in chunks of 256 lights
// (3 float4 per light = the reference's 48-byte `Light`, LightingUtil.hlsl:9-17); every lane reads
// the same LDS address in the light loop (broadcast, conflict-free).
//
// Tiled culling (PBR_FLAG_TILED_CULLING): the tile's world-space AABB comes from wave64
// min/max shuffles plus a 4-entry LDS combine; each chunk's point/spot lights are range-tested
// against it, one light per work-item, and compacted IN ORDER into LDS with a 64-bit ballot +
// mbcnt prefix. A light is dropped only when it is provably beyond the 100-unit range of every
// pixel of the tile, so the reference loop (LightingUtil.hlsl:131) would have added +0 for it:
// the culled result is bit-identical to the unculled one.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pbr_device_math.h"
#include "shade_kernels.h"

namespace pbr {

namespace {

constexpr int kTileW = 32;
constexpr int kTileH = 8;
constexpr int kBlock = kTileW * kTileH;  // 256
constexpr int kChunk = 256;              // lights staged per LDS pass
// Conservative cull radius: d_fp32 >= d_true * (1 - 4.8e-7) (three roundings in L, three in the
// dot, one in sqrt); a margin of 1e-4 relative covers that and the fp32 box-distance error.
constexpr float kCullRadius = 100.01f;

struct TileBounds {
    float mn[3], mx[3];
    bool all_finite;
};

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

// Stage lights [begin, begin+count) of the global list into LDS, culled against the tile when CULL.
// Returns the number staged (identical in every work-item). Caller brackets with barriers.
// Each staged record is the 48-byte Light with its unused pad1 (.w of the position float4)
// replaced by the light's fast-path window flag (pbr_device_math.h, light_window_ok).
template <bool CULL>
__device__ __forceinline__ int stage_chunk(const float4* __restrict__ lights, int begin, int count, float4* s_light,
                                           int* s_wave_cnt, const TileBounds& tb, bool cull_enabled,
                                           bool directional) {
    const int tid = threadIdx.x;
    const bool have = tid < count;
    float4 l0 = make_float4(0.f, 0.f, 0.f, 0.f), l1 = l0, l2 = l0;
    if (have) {
        const float4* src = lights + 3 * (begin + tid);
        l0 = src[0];
        l1 = src[1];
        l2 = src[2];
        l2.w = light_window_ok(directional, l1, l2) ? 1.0f : 0.0f;
    }
    if (!CULL) {
        if (have) {
            s_light[3 * tid + 0] = l0;
            s_light[3 * tid + 1] = l1;
            s_light[3 * tid + 2] = l2;
        }
        return count;
    }
    bool keep = have;
    if (have && cull_enabled) {
        float dx = hmax(hmax(tb.mn[0] - l2.x, l2.x - tb.mx[0]), 0.0f);
        float dy = hmax(hmax(tb.mn[1] - l2.y, l2.y - tb.mx[1]), 0.0f);
        float dz = hmax(hmax(tb.mn[2] - l2.z, l2.z - tb.mx[2]), 0.0f);
        keep = (dx * dx + dy * dy + dz * dz) <= kCullRadius * kCullRadius;
    }
    const uint64_t mask = __ballot(keep);
    const int lane = tid & 63, wave = tid >> 6;
    const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (lane == 0) s_wave_cnt[wave] = __popcll(mask);
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const int c = s_wave_cnt[w];
        off += (w < wave) ? c : 0;
        total += c;
    }
    if (keep) {
        const int slot = off + before;
        s_light[3 * slot + 0] = l0;
        s_light[3 * slot + 1] = l1;
        s_light[3 * slot + 2] = l2;
    }
    return total;
}

// One light's term of ComputeLighting: the exact fast path for every lane, then -- only if some lane
// of the wave left the fast-path window -- the compiler's full IEEE sequences for those lanes. Both
// produce the same bits wherever the fast path is taken, so the sum is independent of the choice.
template <int KIND>  // 0 directional, 1 point, 2 spot
__device__ __forceinline__ void accumulate_light(const PixelInvariants& q, f3 pos, const float4* rec, f3& direct) {
    const float4 a = rec[0], b = rec[1], c = rec[2];
    f3 col;
    bool ok = q.fast_ok && c.w != 0.0f;
    bool lit = true;
    if (KIND == 0) col = directional_light<true>(q, a, b, ok);
    else lit = point_or_spot_light<KIND == 2, true>(q, pos, a, b, c, col, ok);
    if (__any(!ok)) {
        if (!ok) {
            bool unused = true;
            if (KIND == 0) col = directional_light<false>(q, a, b, unused);
            else lit = point_or_spot_light<KIND == 2, false>(q, pos, a, b, c, col, unused);
        }
    }
    if (lit) direct = add3(direct, col);
}

}  // namespace

template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL>
__global__ __launch_bounds__(kBlock) void shade_tile_kernel(GBufferArgs gb, PassArgs ps,
                                                            const float4* __restrict__ lights,
                                                            const float4* __restrict__ env,
                                                            float4* __restrict__ out, int64_t out_stride,
                                                            unsigned long long* __restrict__ cull_stats,
                                                            bool exact_only) {
    __shared__ float4 s_light[3 * kChunk];
    __shared__ int s_wave_cnt[kBlock / 64];
    __shared__ float s_bounds[kBlock / 64][6];

    const int tid = threadIdx.x;
    const int x = blockIdx.x * kTileW + (tid & (kTileW - 1));
    const int y = blockIdx.y * kTileH + (tid / kTileW);
    const bool valid = (x < gb.width) && (y < gb.height);
    const int64_t idx = valid ? (int64_t)y * gb.row_stride + x : 0;  // frames are never empty here

    const f3 pos = mk3(gb.plane[0][idx], gb.plane[1][idx], gb.plane[2][idx]);
    const f3 n = mk3(gb.plane[3][idx], gb.plane[4][idx], gb.plane[5][idx]);
    const f3 albedo = mk3(gb.plane[6][idx], gb.plane[7][idx], gb.plane[8][idx]);
    const float metallic = gb.plane[9][idx];
    const float roughness = gb.plane[10][idx];

    // V = normalize(g_CameraPosW - pin.PosW)  (Default.hlsl:53)
    const f3 v = normalize3(mk3(ps.eye[0] - pos.x, ps.eye[1] - pos.y, ps.eye[2] - pos.z));
    f3 f0;
    if (F0_PLANE) {  // Default.hlsl:92
        f0 = mk3(gb.plane[12][idx], gb.plane[13][idx], gb.plane[14][idx]);
    } else {  // F0 = lerp(g_FresnelR0, diffuseAlbedo, metallic)  (Default.hlsl:94-95)
        f0 = mk3(hlerp(ps.fresnel_r0[0], albedo.x, metallic), hlerp(ps.fresnel_r0[1], albedo.y, metallic),
                 hlerp(ps.fresnel_r0[2], albedo.z, metallic));
    }
    PixelInvariants q = make_invariants(n, v, albedo, f0, metallic, roughness);
    q.fast_ok = !exact_only && fast_window_ok(pos, mk3(ps.eye[0], ps.eye[1], ps.eye[2]), n, albedo, f0, metallic,
                                              roughness);

    TileBounds tb;
    bool cull_enabled = false;
    if (CULL) {
        const bool finite = !valid || (isfinite(pos.x) && isfinite(pos.y) && isfinite(pos.z));
        const float big = 3.0e38f;
        float b[6] = {valid ? pos.x : big,  valid ? pos.y : big,  valid ? pos.z : big,
                      valid ? pos.x : -big, valid ? pos.y : -big, valid ? pos.z : -big};
#pragma unroll
        for (int i = 0; i < 3; ++i) b[i] = wave_min(b[i]);
#pragma unroll
        for (int i = 3; i < 6; ++i) b[i] = wave_max(b[i]);
        if ((tid & 63) == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) s_bounds[tid >> 6][i] = b[i];
        }
        // Non-finite positions in the tile disable culling (the reference's NaN/inf behaviour at
        // LightingUtil.hlsl:131 is then reproduced light by light).
        cull_enabled = __syncthreads_and(finite) != 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            tb.mn[i] = fminf(fminf(s_bounds[0][i], s_bounds[1][i]), fminf(s_bounds[2][i], s_bounds[3][i]));
            tb.mx[i] = fmaxf(fmaxf(s_bounds[0][i + 3], s_bounds[1][i + 3]), fmaxf(s_bounds[2][i + 3], s_bounds[3][i + 3]));
        }
    }

    // ComputeLighting (LightingUtil.hlsl:170-200): in-order sum from +0.
    f3 direct = mk3(0.0f, 0.0f, 0.0f);
    int kept_total = 0;

    // Directional lights [0, n_dir): never culled (no range).
    for (int base = 0; base < ps.n_dir; base += kChunk) {
        const int cnt = min(kChunk, ps.n_dir - base);
        __syncthreads();
        stage_chunk<false>(lights, base, cnt, s_light, s_wave_cnt, tb, false, true);
        __syncthreads();
        for (int j = 0; j < cnt; ++j) accumulate_light<0>(q, pos, &s_light[3 * j], direct);
    }
    // Point lights [n_dir, n_dir + n_point), then spot lights.
    const int pt_begin = ps.n_dir, sp_begin = ps.n_dir + ps.n_point, end = sp_begin + ps.n_spot;
    for (int base = pt_begin; base < sp_begin; base += kChunk) {
        const int cnt = min(kChunk, sp_begin - base);
        __syncthreads();
        const int kept = stage_chunk<CULL>(lights, base, cnt, s_light, s_wave_cnt, tb, cull_enabled, false);
        __syncthreads();
        kept_total += kept;
        for (int j = 0; j < kept; ++j) accumulate_light<1>(q, pos, &s_light[3 * j], direct);
    }
    for (int base = sp_begin; base < end; base += kChunk) {
        const int cnt = min(kChunk, end - base);
        __syncthreads();
        const int kept = stage_chunk<CULL>(lights, base, cnt, s_light, s_wave_cnt, tb, cull_enabled, false);
        __syncthreads();
        kept_total += kept;
        for (int j = 0; j < kept; ++j) accumulate_light<2>(q, pos, &s_light[3 * j], direct);
    }
    if (CULL && tid == 0 && cull_stats != nullptr) {
        atomicAdd(&cull_stats[0], (unsigned long long)kept_total);
        atomicAdd(&cull_stats[1], 1ull);
    }

    f3 ambient;
    if (AMBIENT == kAmbientIblDiffuse) {
        // Default.hlsl:141-146: kS = FresnelSchlick(N, V, F0); kD = (1 - kS)(1 - metallic);
        // irradiance = env.Sample(linear-wrap, WorldToSkyUV(N)); ambient = kD * (irradiance * albedo)
        const float cos_theta = hsat(dot3(n, v));
        const float p = pow5(1.0f - cos_theta);
        const f3 ks = mk3(f0.x + q.one_minus_f0.x * p, f0.y + q.one_minus_f0.y * p, f0.z + q.one_minus_f0.z * p);
        const f3 kd = mk3((1.0f - ks.x) * q.one_minus_metal, (1.0f - ks.y) * q.one_minus_metal,
                          (1.0f - ks.z) * q.one_minus_metal);
        float su, sv;
        world_to_sky_uv(n, su, sv);
        const f3 irr = sample_linear_wrap(env, ps.env_w, ps.env_h, su, sv);
        const f3 diffuse = mk3(irr.x * albedo.x, irr.y * albedo.y, irr.z * albedo.z);
        ambient = mk3(kd.x * diffuse.x, kd.y * diffuse.y, kd.z * diffuse.z);
    } else {
        // g_AmbientLight * diffuseAlbedo  (Default.hlsl:150)
        ambient = mk3(ps.ambient[0] * albedo.x, ps.ambient[1] * albedo.y, ps.ambient[2] * albedo.z);
    }
    if (APPLY_AO) {
        const float ao = gb.plane[11][idx];
        ambient = mk3(ambient.x * ao, ambient.y * ao, ambient.z * ao);
    }
    f3 lit = add3(ambient, direct);
    lit = mk3(lit.x / (lit.x + 1.0f), lit.y / (lit.y + 1.0f), lit.z / (lit.z + 1.0f));  // Default.hlsl:153
    if (valid) {
        out[(int64_t)y * out_stride + x] =
            make_float4(powf(lit.x, kInvGamma), powf(lit.y, kInvGamma), powf(lit.z, kInvGamma), ps.opacity);
    }
}

__global__ void decode_env_kernel(const uint16_t* __restrict__ src, float4* __restrict__ dst, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const ushort4 t = reinterpret_cast<const ushort4*>(src)[i];
        // R16G16B16A16_UNORM decode (WICTextureLoader.cpp:312-367): value / 65535
        dst[i] = make_float4((float)t.x / 65535.0f, (float)t.y / 65535.0f, (float)t.z / 65535.0f, (float)t.w / 65535.0f);
    }
}

template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL>
static hipError_t launch_variant(const LaunchArgs& a, hipStream_t stream) {
    dim3 grid((a.gb.width + kTileW - 1) / kTileW, (a.gb.height + kTileH - 1) / kTileH);
    hipLaunchKernelGGL((shade_tile_kernel<AMBIENT, F0_PLANE, APPLY_AO, CULL>), grid, dim3(kBlock), 0, stream, a.gb,
                       a.ps, a.lights, a.env, a.out, a.out_stride, a.cull_stats, a.exact_only);
    return hipGetLastError();
}

template <int AMBIENT, bool F0_PLANE, bool APPLY_AO>
static hipError_t dispatch_cull(const LaunchArgs& a, hipStream_t s) {
    return a.cull ? launch_variant<AMBIENT, F0_PLANE, APPLY_AO, true>(a, s)
                  : launch_variant<AMBIENT, F0_PLANE, APPLY_AO, false>(a, s);
}
template <int AMBIENT, bool F0_PLANE>
static hipError_t dispatch_ao(const LaunchArgs& a, hipStream_t s) {
    return a.apply_ao ? dispatch_cull<AMBIENT, F0_PLANE, true>(a, s) : dispatch_cull<AMBIENT, F0_PLANE, false>(a, s);
}
template <int AMBIENT>
static hipError_t dispatch_f0(const LaunchArgs& a, hipStream_t s) {
    return a.f0_plane ? dispatch_ao<AMBIENT, true>(a, s) : dispatch_ao<AMBIENT, false>(a, s);
}

hipError_t launch_shade(const LaunchArgs& a, hipStream_t stream) {
    if (a.gb.width <= 0 || a.gb.height <= 0) return hipSuccess;
    return a.ambient_mode == kAmbientIblDiffuse ? dispatch_f0<kAmbientIblDiffuse>(a, stream)
                                                : dispatch_f0<kAmbientConstant>(a, stream);
}

hipError_t launch_decode_env(const uint16_t* src, float4* dst, int n_texels, hipStream_t stream) {
    if (n_texels <= 0) return hipSuccess;
    hipLaunchKernelGGL(decode_env_kernel, dim3((n_texels + 255) / 256), dim3(256), 0, stream, src, dst, n_texels);
    return hipGetLastError();
}

}  // namespace pbr
