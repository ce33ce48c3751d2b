// shade_kernels.hip -- gfx950 kernels for the G-buffer shading hot path.
//
// One workgroup = one 64x8-pixel screen tile = 256 work-items = 4 wave64s. Work-item t shades the
// horizontal pixel pair (2*(t%32), 2*(t%32)+1) of tile row t/32, so wave w owns tile rows 2w, 2w+1:
// each plane load is one 8-byte load per lane (two full 256-byte row segments per wave) and each
// pair of RGBA stores covers two 1-KiB row segments. The pair is shaded in packed fp32
// (pbr_device_math_x2.h): every light-loop operation except the transcendental seeds and compares
// issues once for both pixels.
//
// Lights: the pair kernel reads each light record (3 float4 = the reference's 48-byte `Light`,
// LightingUtil.hlsl:9-17) with wave-uniform scalar loads; nothing is staged and the light loop has no
// barrier. Tiled culling (PBR_FLAG_TILED_CULLING) is per wave: the wave's 64x2-pixel world-space box
// (wave64 butterflies), one range test per lane and light, and the ballot of the survivors walked in
// order. A light is dropped only when it is provably beyond the 100-unit range of every pixel of the
// wave, so the reference loop (LightingUtil.hlsl:131) would have added +0 for it: the culled result
// is bit-identical to the unculled one. (The one-pixel kernel below stages lights through LDS and
// culls per workgroup, with an in-order ballot + mbcnt compaction.)
//
// Exact fallback: a pixel whose inputs or intermediates leave the fast-path window for any light is
// flagged; after the fast loop, a block with any flagged pixel re-runs the light loop for those
// pixels with the compiler's full IEEE sequences (scalar, pbr_device_math.h), replacing their sums.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <vector>

#include "pbr_device_math.h"
#include "pbr_device_math_x2.h"
#include "pbr_balanced.h"
#include "shade_kernels.h"

namespace pbr {

#ifndef PBR_WAVE_TIMELINE
#define PBR_WAVE_TIMELINE 0  // development build: per-wave clock stamps of the pair kernels (pbr_debug_wave_timeline)
#endif
#if PBR_WAVE_TIMELINE
// kTlWords per wave (wave = block * 4 + wave in block): [0] HW_ID | XCC_ID << 32, [1] entry, [2] G-buffer pair
// arrived, [3] light loops start, [4] light loops end, [5] stores issued (s_memrealtime, 100 MHz, one clock for
// the whole chip), [6] / [7] s_memtime (shader clock) at entry / at the end. Lane 0 stores them (vector stores).
constexpr int kTlWords = 8;
static __device__ unsigned long long* g_wave_tl;
static __device__ long long g_wave_tl_cap;
#define TL_RT(i_) (tl[i_] = (unsigned long long)__builtin_amdgcn_s_memrealtime())
#define TL_BEGIN()                                                                                           \
    unsigned long long tl[kTlWords];                                                                         \
    TL_RT(1);                                                                                                \
    tl[6] = (unsigned long long)__builtin_amdgcn_s_memtime();                                                \
    tl[0] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                                            \
            ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32)
#define TL_LOADED()                                      \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    TL_RT(2)
#define TL_FLAGS(f_) (tl[0] |= (unsigned long long)(f_) << 48)  // bits 48+: kernel-specific wave flags
#define TL_END(wv_)                                                                     \
    do {                                                                                \
        TL_RT(5);                                                                       \
        tl[7] = (unsigned long long)__builtin_amdgcn_s_memtime();                       \
        const long long w_ = (wv_);                                                     \
        if ((threadIdx.x & 63) == 0 && g_wave_tl != nullptr && w_ < g_wave_tl_cap) {    \
            for (int i_ = 0; i_ < kTlWords; ++i_) g_wave_tl[w_ * kTlWords + i_] = tl[i_]; \
        }                                                                               \
    } while (0)
#else
#define TL_BEGIN()
#define TL_FLAGS(f_)
#define TL_LOADED()
#define TL_RT(i_)
#define TL_END(wv_)
#endif

namespace {

constexpr int kTileW = 64;  // pixels; 32 work-items x 2 pixels
#ifndef PBR_X2_MIN_WAVES
#define PBR_X2_MIN_WAVES 4  // waves per SIMD the packed kernel is register-allocated for
#endif
#ifndef PBR_BAL_WAVES
#define PBR_BAL_WAVES 4  // waves per workgroup of the balanced-list kernels: 4 (one tile) or 1 (one wave of a tile)
#endif
#ifndef PBR_LEAN_MIN_WAVES
#define PBR_LEAN_MIN_WAVES 4  // waves per SIMD the culled lean pair kernel is register-allocated for
#endif
#ifndef PBR_LEAN_TILES
#define PBR_LEAN_TILES 1  // development: 2 = two tiles per wave in the uniform lean kernels (shade_lean_kernel)
#endif
#ifndef PBR_LEAN_UNIFORM_MIN_WAVES
#define PBR_LEAN_UNIFORM_MIN_WAVES 5  // ... and the unculled (uniform-loop) faithful or constant-ambient ones
#endif
// Waves per SIMD of shade_lean_kernel<AMBIENT, .., CULL, FAITHFUL>: five for the uniform loops, whose loads wait on HBM
// latency with too few waves to cover it (config 2: DESIGN.md §5d), where 96 VGPRs hold the loop without scratch (the
// faithful ones park albedo and 1 - metallic in LDS across it, lean_wave); four for the culled loops (the culled walk
// and its survivor masks need ~105-116 VGPRs) and for the exact diffuse-IBL loop (20 B/lane of scratch at 96).
template <int AMBIENT, bool CULL, bool FAITHFUL>
constexpr int lean_min_waves() {
    return CULL || (!FAITHFUL && AMBIENT == kAmbientIblDiffuse) ? PBR_LEAN_MIN_WAVES : PBR_LEAN_UNIFORM_MIN_WAVES;
}
constexpr int kTileH = 8;
constexpr int kBlock = 256;
constexpr int kChunk = 256;  // lights staged per LDS pass
// Conservative cull radius: d_fp32 >= d_true * (1 - 4.8e-7) (three roundings in L, three in the
// dot, one in sqrt); a margin of 1e-4 relative covers that and the fp32 box-distance error.
constexpr float kCullRadius = 100.01f;
// PBR_FLAG_FAITHFUL: the most light terms a pixel's sum may have for the mode's error bound.
constexpr int kFaithfulMaxTerms = 64;

struct TileBounds {
    float mn[3], mx[3];
};

__device__ __forceinline__ float wave_min(float v) { return wave_min_dpp(v); }  // pbr_device_math_x2.h
__device__ __forceinline__ float wave_max(float v) { return wave_max_dpp(v); }

struct Lds {
    union {
        float4 light[3 * kChunk];  // the exact re-pass's staged lights
        struct {                   // the balanced point-light pass (pbr_balanced.h)
            BalancedWaveLds bal[kBlock / 64];        // one exchange region per wave
            float bal_light[6 * kBalLdsStride];      // the pass's point lights (stage_balanced_lights)
        };
    };
    int wave_cnt[kBlock / 64];
    float bounds[kBlock / 64][6];
#if PBR_BAL_PROFILE
    unsigned long long prof[kBlock / 64][16];
#endif
    int kept_sum, geo_waves;  // tiled-culling statistics of the block
    int exact_px;             // pixels of the block the exact path redid
};

// The one-wave workgroups of the balanced kernels (PBR_BAL_WAVES == 1): the wave's exchange region and the pass's
// point lights only (9.3 KiB + the libm tables: 16 workgroups fit a CU's LDS).
struct LdsBal1 {
    BalancedWaveLds bal[1];
    float bal_light[6 * kBalLdsStride];
#if PBR_BAL_PROFILE
    unsigned long long prof[1][16];
#endif
};

// Stage lights [begin, begin+count) of the global list into LDS, culled against the tile when CULL.
// Returns the number staged (identical in every work-item). Caller brackets with barriers.
// Each staged record is the 48-byte Light with its unused pad1 (.w of the position float4)
// replaced by the light's fast-path window flag (pbr_device_math.h, light_window_ok).
template <bool CULL>
__device__ __forceinline__ int stage_chunk(const float4* __restrict__ lights, int begin, int count, Lds& s,
                                           const TileBounds& tb, bool cull_enabled, bool directional) {
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
            s.light[3 * tid + 0] = l0;
            s.light[3 * tid + 1] = l1;
            s.light[3 * tid + 2] = l2;
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
    if (lane == 0) s.wave_cnt[wave] = __popcll(mask);
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const int c = s.wave_cnt[w];
        off += (w < wave) ? c : 0;
        total += c;
    }
    if (keep) {
        const int slot = off + before;
        s.light[3 * slot + 0] = l0;
        s.light[3 * slot + 1] = l1;
        s.light[3 * slot + 2] = l2;
    }
    return total;
}

// Light j's record as uploaded (the reference's 48-byte Light; pbr_set_pass stores the light's
// fast-path window flag in the unused pad1 = .w of the position). The index is wave-uniform, so
// these are scalar loads through the scalar cache: no LDS staging, no barrier.
struct LightRec {
    float4 s, d, p;
};
__device__ __forceinline__ LightRec light_rec(const float4* __restrict__ lights, int j, const PassArgs& ps) {
    j = PBR_BOUNDS(j, ps.n_dir + ps.n_point + ps.n_spot, kBoundsLight);
    return LightRec{lights[3 * j], lights[3 * j + 1], lights[3 * j + 2]};
}
// The light's fast-path window flag (pbr_set_pass writes 1.0f or 0.0f into pad1) as a lane mask, on
// the scalar unit: the record is in SGPRs, so an integer test of its bits needs no VALU compare.
__device__ __forceinline__ m2 light_flag(const LightRec& r) {
    const uint64_t m = (__float_as_uint(r.p.w) << 1) != 0u ? ~0ull : 0ull;
    return m2{m, m};
}
__device__ __forceinline__ float uniform_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
}

// The tiled-culling range test: point/spot light `lp` may be within range of some point of the box `wb`
// (the box distance against the conservative radius kCullRadius).
__device__ __forceinline__ bool light_survives(float4 lp, const TileBounds& wb) {
    const float dx = hmax(hmax(wb.mn[0] - lp.x, lp.x - wb.mx[0]), 0.0f);
    const float dy = hmax(hmax(wb.mn[1] - lp.y, lp.y - wb.mx[1]), 0.0f);
    const float dz = hmax(hmax(wb.mn[2] - lp.z, lp.z - wb.mx[2]), 0.0f);
    return (dx * dx + dy * dy + dz * dz) <= kCullRadius * kCullRadius;
}

// The number of light terms the wave sums under tiled culling: directional lights + the point/spot lights
// that survive its box (one lane per light, the same test as the loop). PBR_FLAG_FAITHFUL's bound counts
// summed terms, so a culled pass with more lights than the bound allows can still run it per wave.
// The survivor masks of lights [base, base + 256) of the range [.., b1): bit l of m[k] = light base + 64 k + l
// may reach the wave's box. The four chunks' position loads are issued together before any test (a dependent load
// per 64 lights left the wave waiting for each in turn: config 4's per-wave term count and culled walk).
__device__ __forceinline__ void survivor_masks(const float4* __restrict__ lights, int base, int b1,
                                               const TileBounds& wb, bool cull_enabled, uint64_t (&m)[4]) {
    const int lane = (int)(threadIdx.x & 63);
    float4 lp[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = base + 64 * k + lane;
        lp[k] = j < b1 && cull_enabled ? lights[3 * j + 2] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = base + 64 * k + lane;
        m[k] = lanes(j < b1 && (!cull_enabled || light_survives(lp[k], wb)));
    }
}

// The survivor masks of the first 256 point lights as wave_light_terms found them, for the culled walk to reuse
// (valid: a pass without spot lights, whose walk over the point lights starts with the same range and box).
struct FirstSurvivors {
    uint64_t m[4];
    bool valid = false;
};
__device__ __forceinline__ int wave_light_terms(const float4* __restrict__ lights, const PassArgs& ps,
                                                const TileBounds& wb, bool cull_enabled,
                                                FirstSurvivors* first = nullptr) {
    const int b0 = ps.n_dir, b1 = ps.n_dir + ps.n_point + ps.n_spot;
    if (!cull_enabled) return b1;
    int total = ps.n_dir;
    for (int base = b0; base < b1; base += 256) {
        uint64_t m[4];
        if (first != nullptr && first->valid && base == b0) {  // found already (lean_wave's early survivors)
            for (int k = 0; k < 4; ++k) m[k] = first->m[k];
        } else {
            survivor_masks(lights, base, b1, wb, true, m);
            if (first != nullptr && base == b0 && ps.n_spot == 0) {
                for (int k = 0; k < 4; ++k) first->m[k] = m[k];
                first->valid = true;
            }
        }
        total += __popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]);
    }
    return total;
}

// ComputeLighting (LightingUtil.hlsl:170-200) for both pixels of the pair on the packed fast path:
// in-order sum from +0; `redo` collects pixels that left the fast-path window for a lit light.
// LEAN (wave-uniform): the wave's pixels satisfy the extra conditions of brdf_x2<true>.
// CULL: wave-level tiled culling. Each round, lane l range-tests point/spot light base + l against
// the wave's own world-space box `wb` (its 64x2 pixels); the ballot of the survivors is walked in
// increasing bit order, so the kept lights are summed in the reference's order. A dropped light is
// one the reference's `d > 100` test (LightingUtil.hlsl:131) rejects for every pixel of the wave, i.e.
// a +0 term: the result is bit-identical to the unculled pass.
// BALANCED (untiled faithful lean waves, ps.balanced): the point lights run through the back-face-rejected,
// wave-balanced lists of pbr_balanced.h (region `bal`; `geo_a` / `geo_b`: the pair's geometry pixels).
template <bool CULL, bool LEAN, bool FAITHFUL = false, bool BALANCED = false>
__device__ __forceinline__ f3x2 lighting_fast(const PixelInvariants2& q, const f3x2& pos, m2 fast_ok,
                                              const float4* __restrict__ lights, const PassArgs& ps,
                                              const TileBounds& wb, bool cull_enabled, m2& redo, int& kept_total,
                                              BalancedWaveLds* bal = nullptr, const float* bal_lights = nullptr,
                                              bool geo_a = false, bool geo_b = false, BalMasks bm = BalMasks{},
                                              unsigned long long* bal_prof = nullptr,
                                              const FirstSurvivors* first = nullptr) {
    f3x2 direct = splat3(0.0f, 0.0f, 0.0f);
    Faithful2 fi{};
    if (FAITHFUL) fi = make_faithful<!CULL>(q);
    // Exact balanced passes have no directional lights (host: PassArgs::balanced == 2): their loop is compiled
    // out there, it was the register peak of that path.
    const int n_dir = BALANCED && !FAITHFUL ? 0 : ps.n_dir;
    for (int j = 0; j < n_dir; ++j) {  // directional: never culled
        PBR_COLD("directional");
        const LightRec r = light_rec(lights, j, ps);
        m2 ok = fast_ok & light_flag(r);
        if (FAITHFUL) {
            directional_faithful_x2<LEAN, !CULL>(q, fi, r.s, r.d, ok, direct);
        } else {
            const f3x2 c = directional_x2<LEAN>(q, r.s, r.d, ok);
            direct = add3(direct, c);  // shadowFactor (1,1,1) * c == c
        }
        redo |= ~ok;
    }
    const int pt_begin = ps.n_dir, sp_begin = ps.n_dir + ps.n_point, end = sp_begin + ps.n_spot;
    // Point lights, then spot lights: one loop each (SPOT is a template constant, so the point loop
    // carries no spot code and no per-light branch on the kind).
    auto run_kind = [&](auto spot_tag, int b0, int b1) {
        constexpr bool SPOT = decltype(spot_tag)::value;
        auto point = [&](int j) {
            const LightRec r = light_rec(lights, j, ps);
            m2 ok = fast_ok & light_flag(r);
            // An unlit light adds +0 in the reference; here its lanes carry +-0 (zero attenuation)
            // when inside the window, and every lane outside it is redone.
            if (FAITHFUL) {
                point_or_spot_faithful_x2<SPOT, LEAN, !CULL>(q, fi, pos, r.s, r.d, r.p, ok, direct);
            } else {
                const f3x2 c = point_or_spot_x2<SPOT, LEAN>(q, pos, r.s, r.d, r.p, ok);
                direct = add3(direct, c);
            }
            redo |= ~ok;
        };
        if (!CULL) {
            for (int j = b0; j < b1; ++j) point(j);
            return;
        }
        for (int base = b0; base < b1; base += 256) {
            uint64_t ms[4];
            if (!SPOT && first != nullptr && first->valid && base == b0) {  // wave_light_terms tested these
                for (int k = 0; k < 4; ++k) ms[k] = first->m[k];
            } else {
                survivor_masks(lights, base, b1, wb, cull_enabled, ms);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint64_t m = ms[k];
                kept_total += __popcll(m);
                while (m) {
                    const int jl = base + 64 * k + __builtin_ctzll(m);
                    m &= m - 1;
                    point(jl);
                }
            }
        }
    };
    // BALANCED passes have no spot lights (host: PassArgs::balanced): nothing reads q or pos after the
    // balanced loop, so the caller can drop them across it.
    if (BALANCED)
        lighting_balanced_points<!FAITHFUL>(q, fi, pos, geo_a, geo_b, bm, *bal, bal_lights, direct, redo, bal_prof);
    else
        run_kind(std::false_type{}, pt_begin, sp_begin);
    if (!BALANCED && end > sp_begin) run_kind(std::true_type{}, sp_begin, end);
    if (FAITHFUL) {
        // The faithful loop's relative bound holds for sums of normal-range values: a nonzero sum
        // outside [2^-100, 2^100] (tiny sums, where underflowed terms -- a spot cone's pow, say -- carry
        // absolute errors of ~2^-149 that are not small relative to the sum; NaN; overflow) is redone
        // exactly. A zero sum (no light reaches the pixel: every N.L or attenuation is 0, exactly as in
        // the reference) is kept; DESIGN.md §2 states the one residue.
        const m2 in_x = eq(direct.x, 0.0f) | (ge(direct.x, 0x1p-100f) & le(direct.x, 0x1p100f));
        const m2 in_y = eq(direct.y, 0.0f) | (ge(direct.y, 0x1p-100f) & le(direct.y, 0x1p100f));
        const m2 in_z = eq(direct.z, 0.0f) | (ge(direct.z, 0x1p-100f) & le(direct.z, 0x1p100f));
        redo |= ~(in_x & in_y & in_z);
    }
    return direct;
}

// The same sum with the compiler's full IEEE sequences, for one pixel (the exact fallback and the
// PBR_FLAG_EXACT_ONLY mode). Every work-item of the block must call it (it stages lights).
template <bool CULL>
__device__ __forceinline__ void lighting_exact(const PixelInvariants& qa, const PixelInvariants& qb, f3 pa, f3 pb,
                                               bool need_a, bool need_b, const float4* __restrict__ lights,
                                               const PassArgs& ps, Lds& s, const TileBounds& tb,
                                               bool cull_enabled, f3& da, f3& db) {
    da = mk3(0.0f, 0.0f, 0.0f);
    db = mk3(0.0f, 0.0f, 0.0f);
    bool unused = true;
    for (int base = 0; base < ps.n_dir; base += kChunk) {
        const int cnt = min(kChunk, ps.n_dir - base);
        __syncthreads();
        stage_chunk<false>(lights, base, cnt, s, tb, false, true);
        __syncthreads();
        for (int j = 0; j < cnt; ++j) {
            const float4* r = &s.light[3 * j];
            if (need_a) da = add3(da, directional_light<false>(qa, r[0], r[1], unused));
            if (need_b) db = add3(db, directional_light<false>(qb, r[0], r[1], unused));
        }
    }
    const int pt_begin = ps.n_dir, sp_begin = ps.n_dir + ps.n_point, end = sp_begin + ps.n_spot;
#pragma unroll 1
    for (int kind = 1; kind <= 2; ++kind) {
        const int b0 = kind == 1 ? pt_begin : sp_begin, b1 = kind == 1 ? sp_begin : end;
        for (int base = b0; base < b1; base += kChunk) {
            const int cnt = min(kChunk, b1 - base);
            __syncthreads();
            const int kept = stage_chunk<CULL>(lights, base, cnt, s, tb, cull_enabled, false);
            __syncthreads();
            for (int j = 0; j < kept; ++j) {
                const float4* r = &s.light[3 * j];
                f3 c;
                if (need_a) {
                    const bool lit = kind == 1 ? point_or_spot_light<false, false>(qa, pa, r[0], r[1], r[2], c, unused)
                                               : point_or_spot_light<true, false>(qa, pa, r[0], r[1], r[2], c, unused);
                    if (lit) da = add3(da, c);
                }
                if (need_b) {
                    const bool lit = kind == 1 ? point_or_spot_light<false, false>(qb, pb, r[0], r[1], r[2], c, unused)
                                               : point_or_spot_light<true, false>(qb, pb, r[0], r[1], r[2], c, unused);
                    if (lit) db = add3(db, c);
                }
            }
        }
    }
}

// The exact re-pass of the pair kernel, per wave: the same per-light functions as lighting_exact (the
// compiler's IEEE sequences, reference order) with the light records read through the scalar cache instead of
// staged in LDS, so that no block barrier is needed -- a wave whose lanes need no re-pass never waits for the
// other waves of its block (the barrier cost ~4% of a wave's life in the balanced kernel). Wave-uniform.
__device__ __forceinline__ void lighting_exact_wave(const PixelInvariants& qa, const PixelInvariants& qb, f3 pa,
                                                    f3 pb, bool need_a, bool need_b, const float4* __restrict__ lights,
                                                    const PassArgs& ps, f3& da, f3& db) {
    da = mk3(0.0f, 0.0f, 0.0f);
    db = mk3(0.0f, 0.0f, 0.0f);
    bool unused = true;
    for (int j = 0; j < ps.n_dir; ++j) {
        const LightRec r = light_rec(lights, j, ps);
        if (need_a) da = add3(da, directional_light<false>(qa, r.s, r.d, unused));
        if (need_b) db = add3(db, directional_light<false>(qb, r.s, r.d, unused));
    }
    const int pt_begin = ps.n_dir, sp_begin = ps.n_dir + ps.n_point, end = sp_begin + ps.n_spot;
    for (int j = pt_begin; j < end; ++j) {
        const LightRec r = light_rec(lights, j, ps);
        const bool spot = j >= sp_begin;
        f3 c;
        if (need_a) {
            const bool lit = spot ? point_or_spot_light<true, false>(qa, pa, r.s, r.d, r.p, c, unused)
                                  : point_or_spot_light<false, false>(qa, pa, r.s, r.d, r.p, c, unused);
            if (lit) da = add3(da, c);
        }
        if (need_b) {
            const bool lit = spot ? point_or_spot_light<true, false>(qb, pb, r.s, r.d, r.p, c, unused)
                                  : point_or_spot_light<false, false>(qb, pb, r.s, r.d, r.p, c, unused);
            if (lit) db = add3(db, c);
        }
    }
}

// The pair's G-buffer values in packed form: element 0 = pixel A, element 1 = pixel B.
struct PairIn {
    f3x2 pos, n, albedo, f0;
    v2 metallic, roughness, ao;
};

template <bool F0_PLANE, bool APPLY_AO>
__device__ __forceinline__ PairIn load_pair(const GBufferArgs& gb, const PassArgs& ps, int64_t ia, int64_t ib,
                                            bool vector_load) {
    v2 v[15];
    if (vector_load) {  // both pixels exist and the pair is 8-byte aligned in every plane
        ia = PBR_BOUNDS_PIXEL(ia, gb.width, gb.height, gb.row_stride, 2, kBoundsGBuffer);
#pragma unroll
        for (int i = 0; i < 15; ++i) {
            if (i == 11 || (i >= 12 && !F0_PLANE)) continue;  // AO: read at the finish (load_ao_pair)
            const float2 t = *reinterpret_cast<const float2*>(gb.plane[i] + ia);
            v[i] = v2{t.x, t.y};
        }
    } else {
        PBR_COLD("scalar_loads");
        ia = PBR_BOUNDS_PIXEL(ia, gb.width, gb.height, gb.row_stride, 1, kBoundsGBuffer);
        ib = PBR_BOUNDS_PIXEL(ib, gb.width, gb.height, gb.row_stride, 1, kBoundsGBuffer);
#pragma unroll
        for (int i = 0; i < 15; ++i) {
            if (i == 11 || (i >= 12 && !F0_PLANE)) continue;  // AO: read at the finish (load_ao_pair)
            v[i] = v2{gb.plane[i][ia], gb.plane[i][ib]};
        }
    }
    PairIn p;
    p.pos = f3x2{v[0], v[1], v[2]};
    p.n = f3x2{v[3], v[4], v[5]};
    p.albedo = f3x2{v[6], v[7], v[8]};
    p.metallic = v[9];
    p.roughness = v[10];
    p.ao = splat(1.0f);  // PBR_FLAG_APPLY_AO: load_ao_pair after the light loop
    if (F0_PLANE) {  // Default.hlsl:92
        p.f0 = f3x2{v[12], v[13], v[14]};
    } else {  // F0 = lerp(g_FresnelR0, diffuseAlbedo, metallic)  (Default.hlsl:94-95): x + s*(y - x)
        p.f0 = f3x2{ps.fresnel_r0[0] + p.metallic * (p.albedo.x - ps.fresnel_r0[0]),
                    ps.fresnel_r0[1] + p.metallic * (p.albedo.y - ps.fresnel_r0[1]),
                    ps.fresnel_r0[2] + p.metallic * (p.albedo.z - ps.fresnel_r0[2])};
    }
    return p;
}

// An optimisation barrier on the pair's raw values: the compiler must assume they changed, so a computation
// from them after this point is not merged with the same computation before it. No instructions.
__device__ __forceinline__ void launder(v2& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void launder(f3x2& x) {
    launder(x.x);
    launder(x.y);
    launder(x.z);
}
[[maybe_unused]] __device__ __forceinline__ void launder(PairIn& p) {
    launder(p.pos);
    launder(p.n);
    launder(p.albedo);
    launder(p.f0);
    launder(p.metallic);
    launder(p.roughness);
    launder(p.ao);
}

// V = normalize(g_CameraPosW - pin.PosW) (Default.hlsl:53) and the BRDF invariants of the pair. In the window
// every component of eye - pos is 0 or >= 2^-44 and |eye - pos| < 2^22, so the exact fast normalize applies
// once |V| >= 2^-30; other pixels take the IEEE sequences.
__device__ __forceinline__ f3x2 pair_view(const PairIn& p, const PassArgs& ps, m2 fast2) {
    const f3x2 ve = f3x2{ps.eye[0] - p.pos.x, ps.eye[1] - p.pos.y, ps.eye[2] - p.pos.z};
    m2 okv = fast2;
    f3x2 v = normalize_x2(ve, okv);
    const bool va_ok = on(okv.x), vb_ok = on(okv.y);
    if (__builtin_expect(!(va_ok && vb_ok), 0)) {
        PBR_COLD("v_ieee");
        const f3 v0 = va_ok ? lane(v, 0) : normalize3(lane(ve, 0)), v1 = vb_ok ? lane(v, 1) : normalize3(lane(ve, 1));
        v = f3x2{v2{v0.x, v1.x}, v2{v0.y, v1.y}, v2{v0.z, v1.z}};
    }
    return v;
}
__device__ __forceinline__ PixelInvariants2 pair_invariants(const PairIn& p, const PassArgs& ps, m2 fast2) {
    return make_invariants(p.n, pair_view(p, ps, fast2), p.albedo, p.f0, p.metallic, p.roughness, fast2);
}
// Only what the finish reads (make_finish_invariants): the wave-balanced kernels after their light loop.
[[maybe_unused]] __device__ __forceinline__ PixelInvariants2 pair_finish_invariants(const PairIn& p, const PassArgs& ps, m2 fast2) {
    return make_finish_invariants(p.n, pair_view(p, ps, fast2), p.albedo, p.f0, p.metallic);
}

// Ambient + tonemap + gamma for one pixel (Default.hlsl:139-160), returns the output RGBA.
// Reinhard c / (c + 1) (Default.hlsl:153, Skybox.hlsl:47): the Markstein step when `fast` and c is 0 or
// in [2^-100, 2^60] (then c + 1 is in [1, 2^60]); the IEEE division otherwise.
__device__ __forceinline__ float reinhard(float c, bool fast) {
    if (fast && (c == 0.0f || (c >= 0x1p-100f && c <= 0x1p60f))) return div_nr(c, recip_nr(c + 1.0f));
    return c / (c + 1.0f);
}
// PBR_FLAG_FAITHFUL waves: Reinhard with the hardware reciprocal (c >= 0 here; inf / NaN give NaN as
// the IEEE quotient does) and the gamma encode of pow_inv_gamma_faithful.
__device__ __forceinline__ float reinhard_faithful(float c) { return c * __builtin_amdgcn_rcpf(c + 1.0f); }

// The ambient term of Default.hlsl:139-150 (before the AO extension).
template <int AMBIENT>
__device__ __forceinline__ f3 ambient_term(const PixelInvariants& p, const PassArgs& ps, const float4* __restrict__ env) {
    const PixelInvariants& q = p;
    if (AMBIENT == kAmbientIblDiffuse) {
        // Default.hlsl:141-146: kS = FresnelSchlick(N, V, F0); kD = (1 - kS)(1 - metallic);
        // irradiance = env.Sample(linear-wrap, WorldToSkyUV(N)); ambient = kD * (irradiance * albedo)
        const float cos_theta = hsat(dot3(p.n, q.v));
        const float pw = pow5_glibc(1.0f - cos_theta);
        const f3 ks = mk3(p.f0.x + q.one_minus_f0.x * pw, p.f0.y + q.one_minus_f0.y * pw, p.f0.z + q.one_minus_f0.z * pw);
        const f3 kd = mk3((1.0f - ks.x) * q.one_minus_metal, (1.0f - ks.y) * q.one_minus_metal,
                          (1.0f - ks.z) * q.one_minus_metal);
        float su, sv;
        world_to_sky_uv(p.n, su, sv);
        const f3 irr = sample_linear_wrap(env, ps.env_w, ps.env_h, su, sv);
        const f3 diffuse = mk3(irr.x * p.albedo.x, irr.y * p.albedo.y, irr.z * p.albedo.z);
        return mk3(kd.x * diffuse.x, kd.y * diffuse.y, kd.z * diffuse.z);
    }
    // g_AmbientLight * diffuseAlbedo  (Default.hlsl:150)
    return mk3(ps.ambient[0] * p.albedo.x, ps.ambient[1] * p.albedo.y, ps.ambient[2] * p.albedo.z);
}

// The diffuse-IBL ambient of Default.hlsl:141-146 for both pixels of the pair in packed form: ambient_term's
// operations element for element (FresnelSchlick(N, V) with kD = (1 - kS)(1 - metallic), WorldToSkyUV through the
// branch-free pair forms of glibc's atan2f / asinf (libm_f32_x2.h, bit-identical), the linear-wrap env fetch per
// pixel, kD * irradiance * albedo). Faithful waves take the IBL Fresnel x^5 from pow5_faithful (<= 1 ulp from glibc
// off the grazing band x > 0.99, where it is glibc's: <= 1.2e-6 on kD); exact waves glibc's powf.
// Pixels whose normal has a component the pair forms do not cover (NaN, inf, nonzero magnitudes outside
// [2^-40, 2^40], |N.y| > 1) take the scalar functions. `live_a` / `live_b`: the elements whose result is used.
__device__ __forceinline__ f3x2 ambient_ibl_pair(const PixelInvariants2& q, const PassArgs& ps,
                                               const float4* __restrict__ env, bool faithful, bool live_a,
                                               bool live_b) {
    const v2 x = 1.0f - dot3_sat(q.n, q.v);  // 1 - saturate(dot(N, V)): the clamp bit maps NaN to 0 as hsat
    const v2 pw = faithful ? pow5_faithful(x, lanes(live_a || live_b)) : v2{pow5_glibc(x.x), pow5_glibc(x.y)};
    const f3x2 kd = f3x2{(1.0f - (q.f0.x + q.one_minus_f0.x * pw)) * q.one_minus_metal,
                         (1.0f - (q.f0.y + q.one_minus_f0.y * pw)) * q.one_minus_metal,
                         (1.0f - (q.f0.z + q.one_minus_f0.z * pw)) * q.one_minus_metal};
    // WorldToSkyUV (LightingUtil.hlsl:216-225)
    int sa[2], sb[2];
    v2 ux = pbr_atan2f_x2(q.n.z, q.n.x, sa, PBR_LIBM_ATAN_TAB);
    v2 uy = pbr_asinf_x2(q.n.y, sb);
    const bool spec_a = live_a && (sa[0] | sb[0]), spec_b = live_b && (sa[1] | sb[1]);
    if (__builtin_expect(lanes(spec_a || spec_b) != 0, 0)) {
        PBR_COLD("ibl_special");
        if (spec_a) {
            ux.x = pbr_atan2f(q.n.z.x, q.n.x.x);
            uy.x = pbr_asinf(q.n.y.x);
        }
        if (spec_b) {
            ux.y = pbr_atan2f(q.n.z.y, q.n.x.y);
            uy.y = pbr_asinf(q.n.y.y);
        }
    }
    ux = ux * 0.1591f;
    uy = uy * 0.3183f;
    ux = ux + 0.5f;
    uy = uy + 0.5f;
    uy = 1.0f - uy;
    ux = 1.0f - ux;
    ux = ux + 0.25f;
    const f3 ia = sample_linear_wrap(env, ps.env_w, ps.env_h, ux.x, uy.x);
    const f3 ib = sample_linear_wrap(env, ps.env_w, ps.env_h, ux.y, uy.y);
    const f3x2 irr = f3x2{v2{ia.x, ib.x}, v2{ia.y, ib.y}, v2{ia.z, ib.z}};
    return f3x2{kd.x * (irr.x * q.albedo.x), kd.y * (irr.y * q.albedo.y), kd.z * (irr.z * q.albedo.z)};
}

// The finish of both pixels of the pair (finish_pixel each): with the diffuse IBL, the ambient pair is formed in
// packed form first (ambient_ibl_pair); `live_a` / `live_b` say which elements are shaded geometry.
template <int AMBIENT, bool APPLY_AO>
__device__ __forceinline__ void finish_pair(const PixelInvariants2& q2, const PixelInvariants& ua,
                                            const PixelInvariants& ub, float ao_a, float ao_b, f3 da, f3 db,
                                            const PassArgs& ps, const float4* __restrict__ env, bool fast_a,
                                            bool fast_b, bool faithful, bool live_a, bool live_b, float4& ca,
                                            float4& cb);

// The rest of the PS from the ambient term: AO (extension), + direct, Reinhard, gamma (Default.hlsl:150-160).
template <bool APPLY_AO>
__device__ __forceinline__ float4 finish_lit(f3 ambient, float ao, f3 direct, const PassArgs& ps, bool fast,
                                             bool faithful) {
    if (APPLY_AO) ambient = mk3(ambient.x * ao, ambient.y * ao, ambient.z * ao);
    f3 lit = add3(ambient, direct);
    if (faithful) {  // wave-uniform
        lit = mk3(reinhard_faithful(lit.x), reinhard_faithful(lit.y), reinhard_faithful(lit.z));
        return make_float4(pow_inv_gamma_faithful(lit.x), pow_inv_gamma_faithful(lit.y),
                           pow_inv_gamma_faithful(lit.z), ps.opacity);
    }
    PBR_PHASE("xfinish");  // the exact finish (the faithful census stops here)
    lit = mk3(reinhard(lit.x, fast), reinhard(lit.y, fast), reinhard(lit.z, fast));  // Default.hlsl:153
    return make_float4(pow_inv_gamma(lit.x), pow_inv_gamma(lit.y), pow_inv_gamma(lit.z),
                       ps.opacity);
}

template <int AMBIENT, bool APPLY_AO>
__device__ __forceinline__ void finish_pair(const PixelInvariants2& q2, const PixelInvariants& ua,
                                            const PixelInvariants& ub, float ao_a, float ao_b, f3 da, f3 db,
                                            const PassArgs& ps, const float4* __restrict__ env, bool fast_a,
                                            bool fast_b, bool faithful, bool live_a, bool live_b, float4& ca,
                                            float4& cb) {
    if constexpr (AMBIENT == kAmbientIblDiffuse) {
        PBR_PHASE("ibl");
        const f3x2 amb = ambient_ibl_pair(q2, ps, env, faithful, live_a, live_b);
        PBR_PHASE("finish");
        if (live_a) ca = finish_lit<APPLY_AO>(lane(amb, 0), ao_a, da, ps, fast_a, faithful);
        if (live_b) cb = finish_lit<APPLY_AO>(lane(amb, 1), ao_b, db, ps, fast_b, faithful);
    } else {
        if (live_a) ca = finish_lit<APPLY_AO>(ambient_term<AMBIENT>(ua, ps, env), ao_a, da, ps, fast_a, faithful);
        if (live_b) cb = finish_lit<APPLY_AO>(ambient_term<AMBIENT>(ub, ps, env), ao_b, db, ps, fast_b, faithful);
    }
}

template <int AMBIENT, bool APPLY_AO>
__device__ __forceinline__ float4 finish_pixel(const PixelInvariants& p, float ao, f3 direct, const PassArgs& ps,
                                               const float4* __restrict__ env, bool fast, bool faithful = false) {
    return finish_lit<APPLY_AO>(ambient_term<AMBIENT>(p, ps, env), ao, direct, ps, fast, faithful);
}

// The sky pass for a background pixel (Skybox.hlsl:37-49): sampleCoord = normalize(PosW);
// WorldToSkyUV; g_SkyArray[0].Sample(linear-wrap); Reinhard; gamma; alpha 1. sky_colour is the sampled colour,
// sky_finish the rest.
__device__ __forceinline__ f3 sky_colour(f3 dir, const PassArgs& ps, const float4* __restrict__ sky) {
    const f3 c = normalize3(dir);
    float u, v;
    world_to_sky_uv(c, u, v);
    return sample_linear_wrap(sky, ps.sky_w, ps.sky_h, u, v);
}
__device__ __forceinline__ float4 sky_finish(f3 col, bool fast) {
    col = mk3(reinhard(col.x, fast), reinhard(col.y, fast), reinhard(col.z, fast));
    return make_float4(pow_inv_gamma(col.x), pow_inv_gamma(col.y), pow_inv_gamma(col.z),
                       1.0f);
}
__device__ __forceinline__ float4 sky_pixel(f3 dir, const PassArgs& ps, const float4* __restrict__ sky, bool fast) {
    PBR_COLD("sky");
    return sky_finish(sky_colour(dir, ps, sky), fast);
}

// D3D FLOAT -> UNORM8 (the R8G8B8A8_UNORM back buffer, d3dApp.h:124): NaN -> 0, clamp to [0, 1],
// c * 255 + 0.5 in fp32 (no contraction), truncate.
__device__ __forceinline__ uint32_t unorm8(float c) {
    if (!(c == c)) return 0u;
    c = c > 1.0f ? 1.0f : c;
    c = c < 0.0f ? 0.0f : c;
    return (uint32_t)(c * 255.0f + 0.5f);
}

__device__ __forceinline__ void store_pixel(const FrameArgs& fr, int64_t off, float4 c) {
    off = PBR_BOUNDS_PIXEL(off, fr.width, fr.height, fr.out_stride, 1, kBoundsOutput);
    if (fr.format == kOutRgba8) {
        static_cast<uint32_t*>(fr.out)[off] = unorm8(c.x) | (unorm8(c.y) << 8) | (unorm8(c.z) << 16) | (unorm8(c.w) << 24);
    } else {
        static_cast<float4*>(fr.out)[off] = c;
    }
}

// PBR_FLAG_ALPHA_TEST, the reference's ALPHA_TEST permutation (Default.hlsl:111-113, alphaTestedPS): fragOpacity is
// the pixel's opacity-map value (G-buffer plane 15, index gidx) and clip(fragOpacity - 0.1f) discards the fragment
// when that is negative (NaN is not) -- the pixel's output is then left untouched; otherwise fragOpacity is the
// output alpha (Default.hlsl:160). Geometry pixels only (the sky PS has no clip). Returns whether to store.
__device__ __forceinline__ bool alpha_keep(const GBufferArgs& gb, int64_t gidx, float4& c) {
    if (!gb.alpha_test) return true;  // uniform
    const float op = gb.plane[15][PBR_BOUNDS_PIXEL(gidx, gb.width, gb.height, gb.row_stride, 1, kBoundsGBuffer)];
    if (op - 0.1f < 0.0f) return false;
    c.w = op;
    return true;
}

// alpha_keep for the pixel pair at G-buffer row offset `grow` (ga / gb_: geometry), in one uniform branch that
// passes without the flag: the stores of an ordinary pass see no extra work or live values.
__device__ __forceinline__ void alpha_keep_pair(const GBufferArgs& gb, int64_t grow, bool ga, bool gb_, float4& ca,
                                                float4& cb, bool& keep_a, bool& keep_b) {
    keep_a = keep_b = true;
    if (__builtin_expect(gb.alpha_test, 0)) {
        PBR_COLD("alpha");
        if (ga) keep_a = alpha_keep(gb, grow, ca);
        if (gb_) keep_b = alpha_keep(gb, grow + 1, cb);
    }
}

// Coverage of a pixel: geometry unless the frame has a coverage plane holding 0 there.
__device__ __forceinline__ bool is_geometry(const FrameArgs& fr, int x, int y) {
    return fr.coverage == nullptr ||
           fr.coverage[PBR_BOUNDS_PIXEL((int64_t)y * fr.coverage_stride + x, fr.width, fr.height, fr.coverage_stride, 1,
                                        kBoundsCoverage)] != 0;
}

// The lane's index in its wave, from the hardware (v_mbcnt) in volatile asm: the compiler can neither CSE it
// with an earlier value nor hoist it, so the pair kernel re-derives its pixel coordinates at the store
// instead of keeping the 64-bit output offset live across the light loops (at the 128-VGPR cap of 4 waves
// per SIMD that offset was spilled to scratch: 8 bytes written and re-read per work-item).
__device__ __forceinline__ int lane_id_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

}  // namespace

// The IEEE light sum of ONE pixel (wave-uniform `q`, `pos`) with the wave's lanes splitting the lights: lane l
// evaluates light base + l (point_or_spot_light / directional_light, the functions lighting_exact_wave calls),
// and the terms are then added in light order from +0 -- directional, point, spot, as the reference's
// ComputeLighting loops (LightingUtil.hlsl:176-199). An unlit light's term is +0, which leaves the sum as it is
// (it starts at +0 and is never -0), exactly as lighting_exact_wave's skipped addition. One evaluation of a
// light's sequence per 64 lights instead of one per light: a wave with a handful of pixels to re-pass finishes
// in a fraction of the serial loop's time (those waves were the stragglers of short launches).
__device__ __forceinline__ f3 lighting_exact_lanes(const PixelInvariants& q, f3 pos, const float4* __restrict__ lights,
                                                   const PassArgs& ps) {
    const int lane = (int)(threadIdx.x & 63);
    const int n = ps.n_dir + ps.n_point + ps.n_spot, sp_begin = ps.n_dir + ps.n_point;
    f3 sum = mk3(0.0f, 0.0f, 0.0f);
    for (int base = 0; base < n; base += 64) {
        const int j = base + lane;
        f3 t = mk3(0.0f, 0.0f, 0.0f);
        bool unused = true;
        if (j < n) {
            const float4 r0 = lights[3 * j], r1 = lights[3 * j + 1], r2 = lights[3 * j + 2];
            if (j < ps.n_dir) {
                t = directional_light<false>(q, r0, r1, unused);
            } else {
                f3 c;
                const bool lit = j >= sp_begin ? point_or_spot_light<true, false>(q, pos, r0, r1, r2, c, unused)
                                               : point_or_spot_light<false, false>(q, pos, r0, r1, r2, c, unused);
                if (lit) t = c;
            }
        }
        const int cnt = min(64, n - base);
        for (int k = 0; k < cnt; ++k) {
            sum.x = sum.x + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t.x), k));
            sum.y = sum.y + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t.y), k));
            sum.z = sum.z + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t.z), k));
        }
    }
    return sum;
}

// One pixel (G-buffer index `idx`) with the compiler's IEEE sequences: V, the BRDF invariants, the light sum in
// the reference's order (lighting_exact_wave: every light, no culling) and the finish (faithful_finish: the
// faithful wave's finish of a re-passed pixel). Wave-uniform call; lanes with !need return zeros.
// LANES: `idx` is wave-uniform and the lanes split the lights (lighting_exact_lanes); otherwise every lane with
// `need` shades its own pixel.
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool LANES>
__device__ __forceinline__ float4 shade_pixel_exact(const GBufferArgs& gb, const PassArgs& ps,
                                                    const float4* __restrict__ lights, const float4* __restrict__ env,
                                                    int64_t idx, bool need, bool faithful_finish) {
    if (!LANES) idx = need ? idx : 0;
    idx = PBR_BOUNDS_PIXEL(idx, gb.width, gb.height, gb.row_stride, 1, kBoundsGBuffer);
    const f3 pos = mk3(gb.plane[0][idx], gb.plane[1][idx], gb.plane[2][idx]);
    const f3 n = mk3(gb.plane[3][idx], gb.plane[4][idx], gb.plane[5][idx]);
    const f3 albedo = mk3(gb.plane[6][idx], gb.plane[7][idx], gb.plane[8][idx]);
    const float metallic = gb.plane[9][idx], roughness = gb.plane[10][idx];
    const float ao = APPLY_AO ? gb.plane[11][idx] : 1.0f;
    // F0 exactly as load_pair forms it (Default.hlsl:92-95).
    const f3 f0 = F0_PLANE ? mk3(gb.plane[12][idx], gb.plane[13][idx], gb.plane[14][idx])
                           : mk3(ps.fresnel_r0[0] + metallic * (albedo.x - ps.fresnel_r0[0]),
                                 ps.fresnel_r0[1] + metallic * (albedo.y - ps.fresnel_r0[1]),
                                 ps.fresnel_r0[2] + metallic * (albedo.z - ps.fresnel_r0[2]));
    const f3 eye = mk3(ps.eye[0], ps.eye[1], ps.eye[2]);
    const PixelInvariants q = make_invariants(n, normalize3(sub3(eye, pos)), albedo, f0, metallic, roughness);
    f3 d, unused;
    if (LANES)
        d = lighting_exact_lanes(q, pos, lights, ps);
    else
        lighting_exact_wave(q, q, pos, pos, need, false, lights, ps, d, unused);
    return finish_pixel<AMBIENT, APPLY_AO>(q, ao, d, ps, env, false, faithful_finish);
}

// A wave re-passes up to this many pixels one at a time with the lanes splitting the lights (each costs about
// one light's IEEE sequence plus the ordered adds); more, and every lane takes its own pixels.
constexpr int kLanesRepassMax = 8;

// The exact re-pass of one wave's pixels (need_a / need_b: the pair's elements), after the wave has stored
// everything else: each pixel is read back from the G-buffer and evaluated with the IEEE sequences
// (shade_pixel_exact; `faithful`: the finish of a faithful wave), so nothing of the fast path is live here.
// Up to kLanesRepassMax pixels go one at a time with the lanes splitting the lights; more, and every lane
// takes its own pixels.
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO>
__device__ __forceinline__ void repass_exact(const GBufferArgs& gb, const PassArgs& ps,
                                             const float4* __restrict__ lights, const float4* __restrict__ env,
                                             const FrameArgs& fr, int tile_x, int tile_y, int wave_id, bool need_a,
                                             bool need_b, int n_exact, bool faithful) {
    const int tid = threadIdx.x & 63;
    if (n_exact <= kLanesRepassMax) {
        uint64_t ma = lanes(need_a), mb = lanes(need_b);
        while ((ma | mb) != 0) {
            const bool second = ma == 0;
            uint64_t& m = second ? mb : ma;
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const int rx = tile_x * kTileW + 2 * (l & 31) + (second ? 1 : 0);
            const int ry = tile_y * kTileH + 2 * wave_id + (l >> 5);
            float4 c = shade_pixel_exact<AMBIENT, F0_PLANE, APPLY_AO, true>(gb, ps, lights, env,
                                                                            (int64_t)ry * gb.row_stride + rx, true,
                                                                            faithful);
            if (tid == 0 && alpha_keep(gb, (int64_t)ry * gb.row_stride + rx, c))
                store_pixel(fr, (int64_t)ry * fr.out_stride + rx, c);
        }
    } else {
        const int ln = lane_id_fresh();
        const int rx = tile_x * kTileW + 2 * (ln & 31);
        const int ry = tile_y * kTileH + 2 * wave_id + (ln >> 5);
        const int64_t gi = (int64_t)ry * gb.row_stride + rx, oi = (int64_t)ry * fr.out_stride + rx;
        if (lanes(need_a) != 0) {
            float4 c = shade_pixel_exact<AMBIENT, F0_PLANE, APPLY_AO, false>(gb, ps, lights, env, gi, need_a, faithful);
            if (need_a && alpha_keep(gb, gi, c)) store_pixel(fr, oi, c);
        }
        if (lanes(need_b) != 0) {
            float4 c = shade_pixel_exact<AMBIENT, F0_PLANE, APPLY_AO, false>(gb, ps, lights, env, gi + 1, need_b,
                                                                             faithful);
            if (need_b && alpha_keep(gb, gi + 1, c)) store_pixel(fr, oi + 1, c);
        }
    }
}

// BAL (untiled only; PassArgs::balanced): the variant whose lean waves take the wave-balanced point-light lists
// (pbr_balanced.h) -- 1: faithful passes, 2: exact passes; separate instantiations so that the other variants'
// register allocation is untouched. With PBR_BAL_WAVES == 1 the balanced variants run one wave per workgroup
// (blockIdx.y = 4 * tile row + wave, as shade_lean_kernel), each staging the lights itself.
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL, int BAL = 0>
__global__ __launch_bounds__(BAL != 0 && PBR_BAL_WAVES == 1 ? 64 : kBlock, PBR_X2_MIN_WAVES) void shade_tile_kernel(
    GBufferArgs gb, PassArgs ps, const float4* __restrict__ lights, const float4* __restrict__ env, FrameArgs fr,
    int32_t* __restrict__ tile_kept, bool exact_only) {
    constexpr bool kOneWave = BAL != 0 && PBR_BAL_WAVES == 1;
    __shared__ std::conditional_t<kOneWave, LdsBal1, Lds> s;
    TL_BEGIN();
    PBR_PHASE("entry");
#if PBR_BAL_PROFILE
    const long long t_entry = (long long)__builtin_amdgcn_s_memtime();
    unsigned long long* bal_prof = s.prof[__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6];
    if ((threadIdx.x & 63) < 16) bal_prof[threadIdx.x & 63] = 0;
#endif
    load_libm_tables<AMBIENT == kAmbientIblDiffuse>();  // powf (+ atanf with IBL) tables -> LDS (pbr_device_math.h)
    if constexpr (BAL != 0)
        stage_balanced_lights<kOneWave ? 64 : kBlock>(lights, ps.n_dir, ps.n_dir + ps.n_point, s.bal_light,
                                                      BAL == 2 ? 4.0f : 1.0f);
    __syncthreads();
    PBR_PHASE("load_window");

    // wave_id: the wave's two rows of the tile (wave-uniform, SGPR); wslot: its exchange region in this workgroup.
    const int wave_id = kOneWave ? (int)(blockIdx.y & 3) : __builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6;
    const int wslot = kOneWave ? 0 : wave_id;
    const int tile_y = kOneWave ? (int)(blockIdx.y >> 2) : (int)blockIdx.y;
    const int tid = kOneWave ? 64 * wave_id + (int)threadIdx.x : (int)threadIdx.x;
    const int xa = blockIdx.x * kTileW + 2 * (tid & 31);
    const int y = tile_y * kTileH + (tid >> 5);
    const bool va = (xa < gb.width) && (y < gb.height);
    const bool vb = (xa + 1 < gb.width) && (y < gb.height);
    const int64_t row = (int64_t)y * gb.row_stride;
    // Geometry (PS) or background (sky pass) per pixel; background pixels take no part in the tile
    // bounds, the exact re-pass or the lighting (a block without geometry skips it).
    const bool ga = va && is_geometry(fr, xa, y), gb_ = vb && is_geometry(fr, xa + 1, y);
    const bool wave_geometry = lanes(ga || gb_) != 0;  // waves wholly outside the frame skip lighting

    PairIn p = load_pair<F0_PLANE, APPLY_AO>(gb, ps, va ? row + xa : 0, vb ? row + xa + 1 : 0,
                                             vb && gb.pairs_aligned);
    const f3 pa = lane(p.pos, 0), pb = lane(p.pos, 1);

    const bool ok_a = !exact_only && ps.eye_ok && fast_window_ok(pa, lane(p.n, 0), lane(p.albedo, 0), lane(p.f0, 0),
                                                    p.metallic.x, p.roughness.x);
    const bool ok_b = !exact_only && ps.eye_ok && fast_window_ok(pb, lane(p.n, 1), lane(p.albedo, 1), lane(p.f0, 1),
                                                    p.metallic.y, p.roughness.y);
    const m2 fast2 = mask2(ok_a, ok_b);
    TL_LOADED();

    // The pair's invariants. Balanced variants form them on each path that needs them (their balanced paths build
    // their own after pass 1, so computing them here left one dead pair_invariants on the common path); the
    // uniform and culled variants form them here (formed per path, the max-ILP build spilled 20-36 B/lane).
    PixelInvariants2 q2;
    if constexpr (BAL == 0) q2 = pair_invariants(p, ps, fast2);
    auto form_q2 = [&]() {
        if constexpr (BAL != 0) q2 = pair_invariants(p, ps, fast2);
    };

    // The wave's world-space box (its 64x2 pixels; background pixels excluded): wave64 butterflies,
    // then scalar registers. Non-finite positions disable culling for the wave (the reference's
    // NaN/inf behaviour at LightingUtil.hlsl:131 is then reproduced light by light).
    TileBounds wb{};
    bool cull_enabled = false;
    if (CULL) {
        const bool finite = (!ga || (isfinite(pa.x) && isfinite(pa.y) && isfinite(pa.z))) &&
                            (!gb_ || (isfinite(pb.x) && isfinite(pb.y) && isfinite(pb.z)));
        const float big = 3.0e38f;
        wb.mn[0] = uniform_f(wave_min(fminf(ga ? pa.x : big, gb_ ? pb.x : big)));
        wb.mn[1] = uniform_f(wave_min(fminf(ga ? pa.y : big, gb_ ? pb.y : big)));
        wb.mn[2] = uniform_f(wave_min(fminf(ga ? pa.z : big, gb_ ? pb.z : big)));
        wb.mx[0] = uniform_f(wave_max(fmaxf(ga ? pa.x : -big, gb_ ? pb.x : -big)));
        wb.mx[1] = uniform_f(wave_max(fmaxf(ga ? pa.y : -big, gb_ ? pb.y : -big)));
        wb.mx[2] = uniform_f(wave_max(fmaxf(ga ? pa.z : -big, gb_ ? pb.z : -big)));
        cull_enabled = lanes(!finite) == 0;
    }

    // ComputeLighting (LightingUtil.hlsl:170-200) on the packed fast path. From here on the pair
    // lives only in packed form (q2, pos2); the scalar views are rebuilt from it afterwards so the
    // loop does not carry two copies of the invariants.
    int kept_total = 0;
    int bal_items = -1;  // wave-uniform: the balanced pass's live point-light items (statistics), -1 = not run
    m2 redo = m2{0, 0};
    f3x2 pos2 = p.pos;
    f3x2 d2 = splat3(0.0f, 0.0f, 0.0f);
    bool faithful_wave = false;  // wave-uniform: the faithful loop ran, so the finish may be faithful too
    TL_RT(3);
    if (wave_geometry) {  // wave-uniform
        // Wave-uniform choice of the light loop.
        const v2 nn = dot3(p.n, p.n);
        const bool lean_lane = ok_a && ok_b && nn.x <= 1.0f + 0x1p-20f && nn.y <= 1.0f + 0x1p-20f &&
                               f0_nonzero(lane(p.f0, 0)) && f0_nonzero(lane(p.f0, 1));  // make_invariants' f0_nonzero
        // PBR_FLAG_FAITHFUL (host-validated: strengths, ambient and env texels >= 0): in a wave inside the
        // fast window whose albedo is >= 0 and F0 in [0, 1] every light's contribution is >= 0, which bounds
        // the error of the faithful divisions in the sum (brdf_faithful_x2). ps.faithful == 2: a culled pass
        // with more lights than the bound's 64 summed terms, counted per wave here.
        const bool faithful_lane =
            ps.faithful && ok_a && ok_b && p.albedo.x.x >= 0.0f && p.albedo.y.x >= 0.0f && p.albedo.z.x >= 0.0f &&
            p.albedo.x.y >= 0.0f && p.albedo.y.y >= 0.0f && p.albedo.z.y >= 0.0f && p.f0.x.x <= 1.0f &&
            p.f0.y.x <= 1.0f && p.f0.z.x <= 1.0f && p.f0.x.y <= 1.0f && p.f0.y.y <= 1.0f && p.f0.z.y <= 1.0f &&
            p.f0.x.x >= 0.0f && p.f0.y.x >= 0.0f && p.f0.z.x >= 0.0f && p.f0.x.y >= 0.0f && p.f0.y.y >= 0.0f &&
            p.f0.z.y >= 0.0f;
        // BAL == 2 kernels shade exact passes only (host: PassArgs::balanced): no faithful code is compiled in.
        faithful_wave = BAL != 2 && ps.faithful && lanes(!faithful_lane) == 0;
        if (CULL && faithful_wave && ps.faithful == 2)
            faithful_wave = wave_light_terms(lights, ps, wb, cull_enabled) <= kFaithfulMaxTerms;
        const bool lean_wave = lanes(!lean_lane) == 0;
        // Untiled faithful waves read rescaled invariants (exact both ways, faithful_scale).
        if (faithful_wave && lean_wave) {
            if constexpr (BAL == 1 && !CULL) {
#if PBR_BAL_PROFILE
                BAL_PROF_ADD(7, (long long)__builtin_amdgcn_s_memtime() - t_entry);
                unsigned long long* prof = s.prof[wslot];
#else
                unsigned long long* prof = nullptr;
#endif
                // Pass 1 on the raw pair; then the scaled invariants for the loop, rebuilt from the raw pair (the
                // q2 above is not used on this path, so it is not live across pass 1); after the loop the
                // unscaled ones once more for the finish. launder() keeps the compiler from merging the
                // rebuilds with the computation above (which would keep q2 live across the loop: it spilled).
                PBR_PHASE("pass1");
                const BalMasks bm = balanced_pass1<false>(p.pos, p.n, ga, gb_, ps.n_point, kBalDistLoFaithful, s.bal[wslot],
                                                   s.bal_light, prof);
                bal_items = wave_live_items(bm);
                PBR_PHASE("invariants");
                launder(p);
                q2 = pair_invariants(p, ps, fast2);
                faithful_scale(q2);
                d2 = lighting_fast<false, true, true, true>(q2, p.pos, fast2, lights, ps, wb, cull_enabled, redo,
                                                            kept_total, &s.bal[wslot], s.bal_light, ga, gb_, bm,
                                                            prof);
#if PBR_BAL_PROFILE
                const long long t_l1 = (long long)__builtin_amdgcn_s_memtime();
#endif
                PBR_PHASE("invariants2");
                launder(p);
                q2 = pair_finish_invariants(p, ps, fast2);  // the rare exact re-pass reads its pixels again
                pos2 = p.pos;
#if PBR_BAL_PROFILE
                const v2 dep = dot3(q2.n, q2.v);
                if (dep.x == 12345.0f) pos2.x.x = 0.5f;
                BAL_PROF_ADD(8, (long long)__builtin_amdgcn_s_memtime() - t_l1);
#endif
            } else {
                form_q2();
                if (!CULL) faithful_scale(q2);
#if PBR_BAL_PROFILE
                const long long t_u0 = (long long)__builtin_amdgcn_s_memtime();
                BAL_PROF_ADD(11, t_u0 - t_entry);
                BAL_PROF_ADD(13, 1);
#endif
                d2 = lighting_fast<CULL, true, true>(q2, pos2, fast2, lights, ps, wb, cull_enabled, redo, kept_total);
                if (!CULL) faithful_unscale(q2);
#if PBR_BAL_PROFILE
                const v2 dep = d2.x + d2.y;
                if (dep.x == 12345.0f) pos2.x.x = 0.5f;
                BAL_PROF_ADD(12, (long long)__builtin_amdgcn_s_memtime() - t_u0);
#endif
            }
        } else if (faithful_wave) {
            PBR_COLD("faithful_nonlean");
            form_q2();
            if (!CULL) faithful_scale(q2);
            d2 = lighting_fast<CULL, false, true>(q2, pos2, fast2, lights, ps, wb, cull_enabled, redo, kept_total);
            if (!CULL) faithful_unscale(q2);
        } else if (lean_wave) {
            PBR_PHASE("xpass1");  // the exact balanced kernel's path (the faithful census stops here)
            if constexpr (BAL == 2 && !CULL) {
#if PBR_BAL_PROFILE
                unsigned long long* prof = s.prof[wslot];
#else
                unsigned long long* prof = nullptr;
#endif
                // Nothing of the raw pair is carried through the loop: it is read from the G-buffer again
                // afterwards (44 B/px). Carrying it spilled (~250 B/px of scratch traffic): the exact loop's
                // temporaries leave no room for it. The offsets are re-derived from the hardware ids
                // (lane_id_fresh) and the memory clobber keeps the compiler from reusing the first load.
                // (Reading it once more after pass 1 too, so that only position and normal live through
                // pass 1, removed the remaining scratch of this path but measured the same.)
                auto reload = [&]() {
                    asm volatile("" ::: "memory");
                    const int rl = lane_id_fresh();
                    const int rx = blockIdx.x * kTileW + 2 * (rl & 31);
                    const int ry = tile_y * kTileH + 2 * wave_id + (rl >> 5);
                    const int64_t rrow = (int64_t)ry * gb.row_stride + rx;
                    p = load_pair<F0_PLANE, APPLY_AO>(gb, ps, va ? rrow : 0, vb ? rrow + 1 : 0,
                                                      vb && gb.pairs_aligned);
                };
                const BalMasks bm = balanced_pass1<true>(p.pos, p.n, ga, gb_, ps.n_point, kBalDistLoExact, s.bal[wslot],
                                                   s.bal_light, prof);
                bal_items = wave_live_items(bm);
                PBR_PHASE("xinvariants");
                q2 = pair_invariants(p, ps, fast2);
                d2 = lighting_fast<false, true, false, true>(q2, p.pos, fast2, lights, ps, wb, cull_enabled, redo,
                                                             kept_total, &s.bal[wslot], s.bal_light, ga, gb_, bm,
                                                             prof);
                PBR_PHASE("xinvariants2");
                reload();
                q2 = pair_invariants(p, ps, fast2);  // the full set: the finish-only one measured slower here (SGPRs)
                pos2 = p.pos;
            } else {
                form_q2();
                d2 = lighting_fast<CULL, true>(q2, pos2, fast2, lights, ps, wb, cull_enabled, redo, kept_total);
            }
        } else {
            PBR_COLD("general");
            form_q2();
            d2 = lighting_fast<CULL, false>(q2, pos2, fast2, lights, ps, wb, cull_enabled, redo, kept_total);
        }
    } else {
        PBR_COLD("background");
        form_q2();  // background only: the sky pass reads N
    }
    TL_RT(4);
    const PixelInvariants ua = unpack_invariants(q2, 0), ub = unpack_invariants(q2, 1);
    f3 da = lane(d2, 0), db = lane(d2, 1);
    const bool need_a = ga && on(redo.x), need_b = gb_ && on(redo.y);
    // Statistics, one record per wave (kStatsPerBlock ints at slot tile * 4 + wave): culling survivors and
    // whether the wave has geometry (culled passes), the pixels it sends to the exact path, and the work the
    // light loops executed for its geometry pixels: light terms evaluated (every light of the pass in the
    // uniform loop, the survivors of the wave's box under culling, the live items of the balanced lists) and
    // the balanced pass-1 back-face tests.
    PBR_PHASE("stats_repass");
    const int n_exact = __popcll(lanes(need_a)) + __popcll(lanes(need_b));
    const int geo_px = __popcll(lanes(ga)) + __popcll(lanes(gb_));
    if ((tid & 63) == 0 && tile_kept != nullptr) {
        const int64_t slot = ((int64_t)tile_y * gridDim.x + blockIdx.x) * (kBlock / 64) + wave_id;
        const int n_ps = CULL ? kept_total : ps.n_point + ps.n_spot;
        const int terms = !wave_geometry ? 0 : bal_items >= 0 ? bal_items + ps.n_dir * geo_px : (ps.n_dir + n_ps) * geo_px;
        int32_t* st = tile_kept + kStatsPerBlock * slot;
        st[kStatCullKept] = CULL && wave_geometry ? kept_total : 0;
        st[kStatCullTiles] = CULL && wave_geometry ? 1 : 0;
        st[kStatExactPixels] = n_exact;
        st[kStatLightTerms] = terms;
        st[kStatGeometryPixels] = geo_px;
        st[kStatBackfaceTests] = wave_geometry && bal_items >= 0 ? ps.n_point * geo_px : 0;
    }
#if PBR_BAL_PROFILE
    const long long t_b0 = (long long)__builtin_amdgcn_s_memtime();
#endif
    // The balanced variants re-pass their pixels after the stores (repass_exact, as shade_lean_kernel): up to
    // kLanesRepassMax pixels one at a time with the lanes splitting the lights, instead of every light for the
    // whole wave here (~50 us for one pixel, which made the few waves that have one the launch's last).
    if (BAL == 0 && n_exact != 0) {  // wave-uniform: rare (edge inputs, EXACT_ONLY)
        PBR_COLD("exact_repass");
        f3 ea, eb;
        lighting_exact_wave(ua, ub, lane(pos2, 0), lane(pos2, 1), need_a, need_b, lights, ps, ea, eb);
        if (need_a) da = ea;
        if (need_b) db = eb;
    }

#if PBR_BAL_PROFILE
    {
        const long long t_b1 = (long long)__builtin_amdgcn_s_memtime();
        BAL_PROF_ADD(BAL ? 6 : 15, t_b1 - t_entry);
        BAL_PROF_ADD(BAL ? 9 : 14, t_b1 - t_b0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int l = threadIdx.x & 63;
        const int64_t wv = ((int64_t)tile_y * gridDim.x + blockIdx.x) * (kBlock / 64) + wave_id;
        if (l < 16 && g_bal_prof_buf != nullptr && wv < (int64_t)(1 << 18)) g_bal_prof_buf[wv * 16 + l] += bal_prof[l];
    }
#endif
    // The output offset re-derived from the hardware ids (lane_id_fresh): same pixel as xa, y above.
    PBR_PHASE("finish_setup");
    const int ln = lane_id_fresh();
    const int sx = blockIdx.x * kTileW + 2 * (ln & 31);
    const int64_t orow = (int64_t)(tile_y * kTileH + 2 * wave_id + (ln >> 5)) * fr.out_stride + sx;
    // PBR_FLAG_APPLY_AO: the AO pair is read only now, for the finish (Default.hlsl:150 ambient * AO): a value
    // loaded at entry would be live across the light loops (it was the one spilled value of the AO kernels).
    float ao_a = 1.0f, ao_b = 1.0f;
    if (APPLY_AO) {
        const int64_t arow = (int64_t)(tile_y * kTileH + 2 * wave_id + (ln >> 5)) * gb.row_stride + sx;
        if (vb && gb.pairs_aligned) {
            const float2 t = *reinterpret_cast<const float2*>(
                gb.plane[11] + PBR_BOUNDS_PIXEL(arow, gb.width, gb.height, gb.row_stride, 2, kBoundsGBuffer));
            ao_a = t.x;
            ao_b = t.y;
        } else {
            if (va) ao_a = gb.plane[11][PBR_BOUNDS_PIXEL(arow, gb.width, gb.height, gb.row_stride, 1, kBoundsGBuffer)];
            if (vb)
                ao_b = gb.plane[11][PBR_BOUNDS_PIXEL(arow + 1, gb.width, gb.height, gb.row_stride, 1, kBoundsGBuffer)];
        }
    }
    float4 ca = make_float4(0.0f, 0.0f, 0.0f, 0.0f), cb = ca;
    const bool live_a = ga && !(BAL != 0 && need_a), live_b = gb_ && !(BAL != 0 && need_b);
    if (lanes(live_a || live_b) != 0)  // wave-uniform
        finish_pair<AMBIENT, APPLY_AO>(q2, ua, ub, ao_a, ao_b, da, db, ps, env, ok_a, ok_b, faithful_wave, live_a,
                                       live_b, ca, cb);
    PBR_PHASE("store");
    if (va && !ga) ca = sky_pixel(ua.n, ps, fr.sky, !exact_only);
    if (vb && !gb_) cb = sky_pixel(ub.n, ps, fr.sky, !exact_only);
    bool keep_a, keep_b;
    alpha_keep_pair(gb, (int64_t)(tile_y * kTileH + 2 * wave_id + (ln >> 5)) * gb.row_stride + sx, ga, gb_, ca,
                    cb, keep_a, keep_b);
    if (va && keep_a && !(BAL != 0 && need_a)) store_pixel(fr, orow, ca);
    if (vb && keep_b && !(BAL != 0 && need_b)) store_pixel(fr, orow + 1, cb);
    if (BAL != 0 && n_exact != 0)  // wave-uniform
        repass_exact<AMBIENT, F0_PLANE, APPLY_AO>(gb, ps, lights, env, fr, blockIdx.x, tile_y, wave_id, need_a, need_b,
                                                  n_exact, faithful_wave);
    TL_END(((long long)tile_y * gridDim.x + blockIdx.x) * (kBlock / 64) + wave_id);
}

// ---- Lean pair kernel ------------------------------------------------------------------------------------------
// shade_tile_kernel's register allocation is the maximum over every path it carries, and its exact re-pass runs
// with the fast path's state (invariants, positions, sums) still live around it. shade_lean_kernel is the same
// per-wave choice of fast loops for uniform-loop passes (no balanced lists) without a sky pass, but it finishes
// and stores every pixel the fast loop settled first, and only then re-passes the pixels the loop sent to the
// exact path, one at a time, reading each back from the G-buffer and evaluating it with the IEEE sequences
// (shade_pixel_exact; the finish of its wave: faithful in a faithful wave). Nothing of the fast path is live
// there, so the rare path does not raise the register peak of the loops, and the faithful-only instantiation
// (FAITHFUL: the pass has PBR_FLAG_FAITHFUL) carries no faithful code in the exact-mode one. Frames and pass
// statistics are bit-identical to shade_tile_kernel's (tests/test_gpu_lean.py).


// One wave's 64x2 pixels: wave wave_id (tile rows 2 wave_id, 2 wave_id + 1) of tile (tile_x, tile_y), statistics
// slot wave_global. The caller has staged the powf tables.
// `pre`: the pair as the caller already loaded it (the two-tile development kernel, PBR_LEAN_TILES), else nullptr.
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL, bool FAITHFUL>
__device__ __forceinline__ void lean_wave(const GBufferArgs& gb, const PassArgs& ps, const float4* __restrict__ lights,
                                          const float4* __restrict__ env, const FrameArgs& fr,
                                          int32_t* __restrict__ tile_kept, int tile_x, int tile_y, int wave_id,
                                          int64_t wave_global, const PairIn* pre = nullptr) {
    TL_BEGIN();
    const int tid = threadIdx.x;
    const int xa = tile_x * kTileW + 2 * (tid & 31);
    const int y = tile_y * kTileH + 2 * wave_id + (tid >> 5);
    const bool va = (xa < gb.width) && (y < gb.height);
    const bool vb = (xa + 1 < gb.width) && (y < gb.height);
    const int geo_px = __popcll(lanes(va)) + __popcll(lanes(vb));
    if (geo_px == 0) {  // wholly outside the frame: nothing to shade, an empty statistics record
        if ((tid & 63) == 0 && tile_kept != nullptr) {
            int32_t* st = tile_kept + kStatsPerBlock * wave_global;
            for (int i = 0; i < kStatsPerBlock; ++i) st[i] = 0;
        }
        return;
    }
    const int64_t row = (int64_t)y * gb.row_stride;
    constexpr bool kPark = lean_min_waves<AMBIENT, CULL, FAITHFUL>() >= 5;
    __shared__ v2 s_park[4][64];   // five-wave kernels' faithful waves: albedo, 1 - metallic across the light loop
    bool need_a, need_b;           // pixels for the IEEE path (the exact re-pass)
    bool faithful_wave = false;    // wave-uniform
    int kept_total = 0;
    {
        // Culled passes without spot lights: the first 256 point lights' positions (lane j: light n_dir + 64 k + j)
        // are loaded before the pair, so the culling box and the survivor tests below overlap the G-buffer loads'
        // latency instead of following it; the survivor masks then serve the term count and the walk. (Issuing them
        // between the position planes and the other planes measured 3.5% slower on config 4: the per-lane choice of
        // load form makes the later planes wait for the light loads.)
        float4 lp[4];
        const bool early = CULL && ps.n_spot == 0 && ps.n_point > 0;  // wave-uniform
        if (CULL && early) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = ps.n_dir + 64 * k + tid;
                lp[k] = j < ps.n_dir + ps.n_point ? lights[3 * PBR_BOUNDS(j, ps.n_dir + ps.n_point, kBoundsLight) + 2]
                                                  : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
        }
        PairIn p = pre != nullptr ? *pre
                                  : load_pair<F0_PLANE, APPLY_AO>(gb, ps, va ? row + xa : 0, vb ? row + xa + 1 : 0,
                                                                  vb && gb.pairs_aligned);
        TileBounds wb{};
        bool cull_enabled = false;
        FirstSurvivors first;  // the first survivor masks, for the faithful term count and the culled walk
        if (CULL) {  // the wave's box, as in shade_pair_wave (every pixel is geometry: no sky pass)
            const f3 pa = lane(p.pos, 0), pb = lane(p.pos, 1);
            const bool finite = (!va || (isfinite(pa.x) && isfinite(pa.y) && isfinite(pa.z))) &&
                                (!vb || (isfinite(pb.x) && isfinite(pb.y) && isfinite(pb.z)));
            const float big = 3.0e38f;
            wb.mn[0] = uniform_f(wave_min(fminf(va ? pa.x : big, vb ? pb.x : big)));
            wb.mn[1] = uniform_f(wave_min(fminf(va ? pa.y : big, vb ? pb.y : big)));
            wb.mn[2] = uniform_f(wave_min(fminf(va ? pa.z : big, vb ? pb.z : big)));
            wb.mx[0] = uniform_f(wave_max(fmaxf(va ? pa.x : -big, vb ? pb.x : -big)));
            wb.mx[1] = uniform_f(wave_max(fmaxf(va ? pa.y : -big, vb ? pb.y : -big)));
            wb.mx[2] = uniform_f(wave_max(fmaxf(va ? pa.z : -big, vb ? pb.z : -big)));
            cull_enabled = lanes(!finite) == 0;
            if (early && cull_enabled) {  // survivor_masks' tests on the preloaded positions
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    first.m[k] = lanes(ps.n_dir + 64 * k + tid < ps.n_dir + ps.n_point && light_survives(lp[k], wb));
                first.valid = true;
            }
        }
        // shade_pair_wave's per-wave choice of the light loop (BAL 0, every pixel geometry), unchanged.
        const bool ok_a = ps.eye_ok && fast_window_ok(lane(p.pos, 0), lane(p.n, 0), lane(p.albedo, 0),
                                                      lane(p.f0, 0), p.metallic.x, p.roughness.x);
        const bool ok_b = ps.eye_ok && fast_window_ok(lane(p.pos, 1), lane(p.n, 1), lane(p.albedo, 1),
                                                      lane(p.f0, 1), p.metallic.y, p.roughness.y);
        const m2 fast2 = mask2(ok_a, ok_b);
        TL_LOADED();
        PixelInvariants2 q2 = pair_invariants(p, ps, fast2);
        const v2 nn = dot3(p.n, p.n);
        const bool lean_lane = ok_a && ok_b && nn.x <= 1.0f + 0x1p-20f && nn.y <= 1.0f + 0x1p-20f &&
                               on(q2.f0_nonzero.x) && on(q2.f0_nonzero.y);
        if (FAITHFUL) {
            const bool faithful_lane =
                ok_a && ok_b && p.albedo.x.x >= 0.0f && p.albedo.y.x >= 0.0f && p.albedo.z.x >= 0.0f &&
                p.albedo.x.y >= 0.0f && p.albedo.y.y >= 0.0f && p.albedo.z.y >= 0.0f && p.f0.x.x <= 1.0f &&
                p.f0.y.x <= 1.0f && p.f0.z.x <= 1.0f && p.f0.x.y <= 1.0f && p.f0.y.y <= 1.0f && p.f0.z.y <= 1.0f &&
                p.f0.x.x >= 0.0f && p.f0.y.x >= 0.0f && p.f0.z.x >= 0.0f && p.f0.x.y >= 0.0f && p.f0.y.y >= 0.0f &&
                p.f0.z.y >= 0.0f;
            faithful_wave = lanes(!faithful_lane) == 0;
            if (CULL && faithful_wave && ps.faithful == 2)
                faithful_wave = wave_light_terms(lights, ps, wb, cull_enabled, &first) <= kFaithfulMaxTerms;
        }
        const bool lean_wave = lanes(!lean_lane) == 0;
        TL_RT(3);
        m2 redo = m2{0, 0};
        f3x2 d2;
        if (faithful_wave) {
            if (!CULL) faithful_scale(q2);
            // Five-wave kernels: albedo and 1 - metallic feed the faithful loop only through make_faithful's hoisted
            // products, but the finish needs them; parked in LDS across the loop (the memory clobber keeps the
            // compiler from forwarding the stored values), they hold no VGPRs there: at the 96-VGPR budget of five
            // waves per SIMD the loop then runs without scratch.
            if constexpr (kPark) {
                const int l = (int)(threadIdx.x & 63);
                s_park[0][l] = q2.albedo.x;
                s_park[1][l] = q2.albedo.y;
                s_park[2][l] = q2.albedo.z;
                s_park[3][l] = q2.one_minus_metal;
                asm volatile("" ::: "memory");
            }
            if (lean_wave)
                d2 = lighting_fast<CULL, true, true>(q2, p.pos, fast2, lights, ps, wb, cull_enabled, redo, kept_total,
                                                     nullptr, nullptr, false, false, BalMasks{}, nullptr, &first);
            else
                d2 = lighting_fast<CULL, false, true>(q2, p.pos, fast2, lights, ps, wb, cull_enabled, redo, kept_total,
                                                      nullptr, nullptr, false, false, BalMasks{}, nullptr, &first);
            if constexpr (kPark) {
                asm volatile("" ::: "memory");
                const int l = lane_id_fresh();
                q2.albedo = f3x2{s_park[0][l], s_park[1][l], s_park[2][l]};
                q2.one_minus_metal = s_park[3][l];
            }
            if (!CULL) faithful_unscale(q2);
        } else if (lean_wave) {
            d2 = lighting_fast<CULL, true>(q2, p.pos, fast2, lights, ps, wb, cull_enabled, redo, kept_total,
                                           nullptr, nullptr, false, false, BalMasks{}, nullptr, &first);
        } else {
            d2 = lighting_fast<CULL, false>(q2, p.pos, fast2, lights, ps, wb, cull_enabled, redo, kept_total,
                                            nullptr, nullptr, false, false, BalMasks{}, nullptr, &first);
        }
        TL_RT(4);
        {
            need_a = va && on(redo.x);
            need_b = vb && on(redo.y);
            // Finish and store every pixel the fast loop settled.
            const PixelInvariants ua = unpack_invariants(q2, 0), ub = unpack_invariants(q2, 1);
            const int ln = lane_id_fresh();
            const int sx = tile_x * kTileW + 2 * (ln & 31);
            const int64_t orow = (int64_t)(tile_y * kTileH + 2 * wave_id + (ln >> 5)) * fr.out_stride + sx;
            float ao_a = 1.0f, ao_b = 1.0f;
            if (APPLY_AO) {
                const int64_t arow = (int64_t)(tile_y * kTileH + 2 * wave_id + (ln >> 5)) * gb.row_stride + sx;
                if (vb && gb.pairs_aligned) {
                    const float2 t = *reinterpret_cast<const float2*>(
                        gb.plane[11] + PBR_BOUNDS_PIXEL(arow, gb.width, gb.height, gb.row_stride, 2, kBoundsGBuffer));
                    ao_a = t.x;
                    ao_b = t.y;
                } else {
                    if (va)
                        ao_a = gb.plane[11][PBR_BOUNDS_PIXEL(arow, gb.width, gb.height, gb.row_stride, 1,
                                                             kBoundsGBuffer)];
                    if (vb)
                        ao_b = gb.plane[11][PBR_BOUNDS_PIXEL(arow + 1, gb.width, gb.height, gb.row_stride, 1,
                                                             kBoundsGBuffer)];
                }
            }
            float4 ca = make_float4(0.0f, 0.0f, 0.0f, 0.0f), cb = ca;
            finish_pair<AMBIENT, APPLY_AO>(q2, ua, ub, ao_a, ao_b, lane(d2, 0), lane(d2, 1), ps, env, ok_a, ok_b,
                                           faithful_wave, va && !need_a, vb && !need_b, ca, cb);
            bool keep_a, keep_b;
            alpha_keep_pair(gb, (int64_t)(tile_y * kTileH + 2 * wave_id + (ln >> 5)) * gb.row_stride + sx,
                            va && !need_a, vb && !need_b, ca, cb, keep_a, keep_b);
            if (va && !need_a && keep_a) store_pixel(fr, orow, ca);
            if (vb && !need_b && keep_b) store_pixel(fr, orow + 1, cb);
        }
    }
    const int n_exact = __popcll(lanes(need_a)) + __popcll(lanes(need_b));
    if ((tid & 63) == 0 && tile_kept != nullptr) {
        const bool culled = CULL;
        const int n_ps = culled ? kept_total : ps.n_point + ps.n_spot;
        int32_t* st = tile_kept + kStatsPerBlock * wave_global;
        st[kStatCullKept] = culled ? kept_total : 0;
        st[kStatCullTiles] = culled ? 1 : 0;
        st[kStatExactPixels] = n_exact;
        st[kStatLightTerms] = (ps.n_dir + n_ps) * geo_px;
        st[kStatGeometryPixels] = geo_px;
        st[kStatBackfaceTests] = 0;
    }
    if (n_exact != 0)  // wave-uniform, rare: the IEEE path
        repass_exact<AMBIENT, F0_PLANE, APPLY_AO>(gb, ps, lights, env, fr, tile_x, tile_y, wave_id, need_a, need_b,
                                                  n_exact, faithful_wave);
    TL_FLAGS((n_exact != 0 ? 1 : 0) | (FAITHFUL && !faithful_wave ? 2 : 0));
    TL_END(wave_global);
}

// One wave per workgroup (blockIdx.y = 4 * tile row + wave): a wave's slot on its SIMD is refilled as soon as it
// ends (with 4-wave workgroups a new workgroup waited for four free slots on the CU). Tried and dropped: a
// persistent grid of 3 or 4 waves per SIMD walking the waves (same-box A/B config 2 0.058 -> 0.090 ms: each wave
// then waits for its own G-buffer loads, which the independent waves overlap).
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL, bool FAITHFUL>
__global__ __launch_bounds__(64, (lean_min_waves<AMBIENT, CULL, FAITHFUL>())) void shade_lean_kernel(GBufferArgs gb, PassArgs ps,
                                                            const float4* __restrict__ lights,
                                                            const float4* __restrict__ env, FrameArgs fr,
                                                            int32_t* __restrict__ tile_kept) {
    // powf tables -> LDS: the exact finish's gamma, spot cones, the faithful gamma's edges (+ atanf rows with IBL)
    load_libm_tables<AMBIENT == kAmbientIblDiffuse>();
    __syncthreads();
#if PBR_LEAN_TILES == 2
    // Development (PBR_LEAN_TILES=2, uniform loops): each wave shades two tiles' 64x2 pixels, tile rows 2t and 2t + 1
    // (blockIdx.y = 4 t + wave), with the second tile's G-buffer pair loaded before the first tile is shaded, so
    // that its loads are in flight under the first tile's light loop.
    if constexpr (!CULL) {
        const int wave_id = blockIdx.y & 3, ty0 = (blockIdx.y >> 2) * 2;
        const int tiles_y = (gb.height + kTileH - 1) / kTileH;
        auto load_tile = [&](int ty) {
            const int xa = blockIdx.x * kTileW + 2 * (threadIdx.x & 31);
            const int y = ty * kTileH + 2 * wave_id + (threadIdx.x >> 5);
            const bool va = (xa < gb.width) && (y < gb.height), vb = (xa + 1 < gb.width) && (y < gb.height);
            const int64_t row = (int64_t)y * gb.row_stride;
            return load_pair<F0_PLANE, APPLY_AO>(gb, ps, va ? row + xa : 0, vb ? row + xa + 1 : 0,
                                                 vb && gb.pairs_aligned);
        };
        const bool has1 = ty0 + 1 < tiles_y;  // uniform
        const PairIn p0 = load_tile(ty0);
        const PairIn p1 = load_tile(has1 ? ty0 + 1 : ty0);
        auto slot = [&](int ty) { return ((int64_t)ty * gridDim.x + blockIdx.x) * (kBlock / 64) + wave_id; };
        lean_wave<AMBIENT, F0_PLANE, APPLY_AO, CULL, FAITHFUL>(gb, ps, lights, env, fr, tile_kept, blockIdx.x, ty0,
                                                               wave_id, slot(ty0), &p0);
        if (has1)
            lean_wave<AMBIENT, F0_PLANE, APPLY_AO, CULL, FAITHFUL>(gb, ps, lights, env, fr, tile_kept, blockIdx.x,
                                                                   ty0 + 1, wave_id, slot(ty0 + 1), &p1);
        return;
    }
#endif
    lean_wave<AMBIENT, F0_PLANE, APPLY_AO, CULL, FAITHFUL>(gb, ps, lights, env, fr, tile_kept, blockIdx.x,
                                                           blockIdx.y >> 2, blockIdx.y & 3,
                                                           ((int64_t)(blockIdx.y >> 2) * gridDim.x + blockIdx.x) *
                                                                   (kBlock / 64) + (blockIdx.y & 3));
}

// ---- One pixel per work-item (32x8 tiles) ---------------------------------------------------------
// The same algorithm on the scalar fast path (pbr_device_math.h). Packing a pixel pair (above) halves
// the instruction count but not the VALU cycles (a v_pk_fma_f32 issues in twice the cycles of a
// v_fma_f32 on gfx950), and its register footprint costs a wave per SIMD; the launcher picks the
// faster layout (PBR_PIXELS_PER_THREAD).
namespace {

constexpr int kTileW1 = 32;

template <bool CULL>
__device__ __forceinline__ f3 lighting_fast1(const PixelInvariants& q, f3 pos, const float4* __restrict__ lights,
                                             const PassArgs& ps, Lds& s, const TileBounds& tb, bool cull_enabled,
                                             bool& redo, int& kept_total) {
    f3 direct = mk3(0.0f, 0.0f, 0.0f);
    for (int base = 0; base < ps.n_dir; base += kChunk) {  // directional: never culled
        const int cnt = min(kChunk, ps.n_dir - base);
        __syncthreads();
        stage_chunk<false>(lights, base, cnt, s, tb, false, true);
        __syncthreads();
        for (int j = 0; j < cnt; ++j) {
            const float4* r = &s.light[3 * j];
            bool ok = q.fast_ok && r[2].w != 0.0f;
            const f3 c = directional_light<true>(q, r[0], r[1], ok);
            redo = redo || !ok;
            direct = add3(direct, c);  // shadowFactor (1,1,1) * c == c
        }
    }
    const int pt_begin = ps.n_dir, sp_begin = ps.n_dir + ps.n_point, end = sp_begin + ps.n_spot;
#pragma unroll 1
    for (int kind = 1; kind <= 2; ++kind) {
        const int b0 = kind == 1 ? pt_begin : sp_begin, b1 = kind == 1 ? sp_begin : end;
        for (int base = b0; base < b1; base += kChunk) {
            const int cnt = min(kChunk, b1 - base);
            __syncthreads();
            const int kept = stage_chunk<CULL>(lights, base, cnt, s, tb, cull_enabled, false);
            __syncthreads();
            kept_total += kept;
            for (int j = 0; j < kept; ++j) {
                const float4* r = &s.light[3 * j];
                bool ok = q.fast_ok && r[2].w != 0.0f;
                f3 c;
                const bool lit = kind == 1 ? point_or_spot_light<false, true>(q, pos, r[0], r[1], r[2], c, ok)
                                           : point_or_spot_light<true, true>(q, pos, r[0], r[1], r[2], c, ok);
                if (lit) {  // an unlit light adds +0 in the reference: the identity on this sum
                    redo = redo || !ok;
                    direct = add3(direct, c);
                }
            }
        }
    }
    return direct;
}

}  // namespace

template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL>
__global__ __launch_bounds__(kBlock) void shade_tile1_kernel(GBufferArgs gb, PassArgs ps,
                                                             const float4* __restrict__ lights,
                                                             const float4* __restrict__ env, FrameArgs fr,
                                                             int32_t* __restrict__ tile_kept,
                                                             bool exact_only) {
    __shared__ Lds s;
    load_libm_tables<AMBIENT == kAmbientIblDiffuse>();  // powf (+ atanf with IBL) tables -> LDS (pbr_device_math.h)
    __syncthreads();
    const int tid = threadIdx.x;
    const int x = blockIdx.x * kTileW1 + (tid & (kTileW1 - 1));
    const int y = blockIdx.y * kTileH + (tid / kTileW1);
    const bool valid = (x < gb.width) && (y < gb.height);
    const int64_t idx = PBR_BOUNDS_PIXEL(valid ? (int64_t)y * gb.row_stride + x : 0, gb.width, gb.height, gb.row_stride,
                                         1, kBoundsGBuffer);  // frames are never empty here
    const bool geom = valid && is_geometry(fr, x, y);
    const bool any_geometry = fr.coverage == nullptr || __syncthreads_or(geom);

    f3 pos, n, albedo, f0;
    pos = mk3(gb.plane[0][idx], gb.plane[1][idx], gb.plane[2][idx]);
    n = mk3(gb.plane[3][idx], gb.plane[4][idx], gb.plane[5][idx]);
    albedo = mk3(gb.plane[6][idx], gb.plane[7][idx], gb.plane[8][idx]);
    const float metallic = gb.plane[9][idx];
    const float roughness = gb.plane[10][idx];
    const float ao = APPLY_AO ? gb.plane[11][idx] : 1.0f;
    if (F0_PLANE) {  // Default.hlsl:92
        f0 = mk3(gb.plane[12][idx], gb.plane[13][idx], gb.plane[14][idx]);
    } else {  // F0 = lerp(g_FresnelR0, diffuseAlbedo, metallic)  (Default.hlsl:94-95)
        f0 = mk3(hlerp(ps.fresnel_r0[0], albedo.x, metallic), hlerp(ps.fresnel_r0[1], albedo.y, metallic),
                 hlerp(ps.fresnel_r0[2], albedo.z, metallic));
    }
    // V = normalize(g_CameraPosW - pin.PosW)  (Default.hlsl:53)
    const f3 eye = mk3(ps.eye[0], ps.eye[1], ps.eye[2]);
    PixelInvariants q = make_invariants(n, normalize3(sub3(eye, pos)), albedo, f0, metallic, roughness);
    q.fast_ok = !exact_only && ps.eye_ok && fast_window_ok(pos, n, albedo, f0, metallic, roughness);

    TileBounds tb{};
    bool cull_enabled = false;
    if (CULL) {
        const bool finite = !geom || (isfinite(pos.x) && isfinite(pos.y) && isfinite(pos.z));
        const float big = 3.0e38f;
        float b[6] = {geom ? pos.x : big,  geom ? pos.y : big,  geom ? pos.z : big,
                      geom ? pos.x : -big, geom ? pos.y : -big, geom ? pos.z : -big};
#pragma unroll
        for (int i = 0; i < 3; ++i) b[i] = wave_min(b[i]);
#pragma unroll
        for (int i = 3; i < 6; ++i) b[i] = wave_max(b[i]);
        if ((tid & 63) == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) s.bounds[tid >> 6][i] = b[i];
        }
        cull_enabled = __syncthreads_and(finite) != 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            tb.mn[i] = fminf(fminf(s.bounds[0][i], s.bounds[1][i]), fminf(s.bounds[2][i], s.bounds[3][i]));
            tb.mx[i] = fmaxf(fmaxf(s.bounds[0][i + 3], s.bounds[1][i + 3]), fmaxf(s.bounds[2][i + 3], s.bounds[3][i + 3]));
        }
    }

    int kept_total = 0;
    bool redo = false;
    f3 direct = mk3(0.0f, 0.0f, 0.0f);
    if (any_geometry) direct = lighting_fast1<CULL>(q, pos, lights, ps, s, tb, cull_enabled, redo, kept_total);
    const bool need = geom && redo;
    const int n_exact = __syncthreads_count(need);
    if (n_exact != 0) {  // block-uniform: rare (edge inputs, EXACT_ONLY)
        f3 e, unused;
        lighting_exact<CULL>(q, q, pos, pos, need, false, lights, ps, s, tb, cull_enabled, e, unused);
        if (need) direct = e;
    }
    const int geo_px = __syncthreads_count(geom);
    if (tid == 0 && tile_kept != nullptr) {  // this layout culls per block (32x8 pixels)
        const int64_t t = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
        int32_t* st = tile_kept + kStatsPerBlock * t;
        st[kStatCullKept] = CULL && any_geometry ? kept_total : 0;
        st[kStatCullTiles] = CULL && any_geometry ? 1 : 0;
        st[kStatExactPixels] = n_exact;
        st[kStatLightTerms] = any_geometry ? (ps.n_dir + (CULL ? kept_total : ps.n_point + ps.n_spot)) * geo_px : 0;
        st[kStatGeometryPixels] = geo_px;
        st[kStatBackfaceTests] = 0;
    }
    if (valid) {
        float4 c = geom ? finish_pixel<AMBIENT, APPLY_AO>(q, ao, direct, ps, env, q.fast_ok)
                        : sky_pixel(q.n, ps, fr.sky, !exact_only);
        if (!geom || alpha_keep(gb, idx, c)) store_pixel(fr, (int64_t)y * fr.out_stride + x, c);
    }
}

// The balanced-list kernels (BAL 1, 2) are compiled in their own translation unit, shade_kernels_bal.hip,
// which includes this file with PBR_BAL_TU defined: the Makefile builds this one with the max-ILP machine
// scheduler (faster for the uniform and culled loops, no scratch) and that one with the default scheduler
// (max-ILP spills 12-44 B/lane in the balanced kernels). Profiling builds (PBR_BAL_PROFILE) keep everything
// here, so that one g_bal_prof_buf collects every kernel's stamps.
#if defined(PBR_BAL_PROFILE) && PBR_BAL_PROFILE
#define PBR_SPLIT_BAL 0
#else
#define PBR_SPLIT_BAL 1
#endif
#ifndef PBR_BAL_TU
#define PBR_BAL_TU 0
#endif

// Launches the balanced variant (a.ps.balanced 1 or 2) of shade_tile_kernel over `grid`.
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO>
hipError_t launch_balanced(const LaunchArgs& a, dim3 grid, hipStream_t stream);

#if PBR_BAL_TU == PBR_SPLIT_BAL
template <int AMBIENT, bool F0_PLANE, bool APPLY_AO>
hipError_t launch_balanced(const LaunchArgs& a, dim3 grid, hipStream_t stream) {
    const dim3 g = PBR_BAL_WAVES == 1 ? dim3(grid.x, grid.y * (kBlock / 64)) : grid;
    const dim3 blk(PBR_BAL_WAVES == 1 ? 64 : kBlock);
    if (a.ps.balanced == 1)
        hipLaunchKernelGGL((shade_tile_kernel<AMBIENT, F0_PLANE, APPLY_AO, false, 1>), g, blk, 0, stream, a.gb, a.ps,
                           a.lights, a.env, a.frame, a.tile_kept, a.exact_only);
    else
        hipLaunchKernelGGL((shade_tile_kernel<AMBIENT, F0_PLANE, APPLY_AO, false, 2>), g, blk, 0, stream, a.gb, a.ps,
                           a.lights, a.env, a.frame, a.tile_kept, a.exact_only);
    return hipGetLastError();
}
#define PBR_INSTANTIATE_BAL(A, F, O) template hipError_t launch_balanced<A, F, O>(const LaunchArgs&, dim3, hipStream_t);
PBR_INSTANTIATE_BAL(kAmbientConstant, false, false)
PBR_INSTANTIATE_BAL(kAmbientConstant, false, true)
PBR_INSTANTIATE_BAL(kAmbientConstant, true, false)
PBR_INSTANTIATE_BAL(kAmbientConstant, true, true)
PBR_INSTANTIATE_BAL(kAmbientIblDiffuse, false, false)
PBR_INSTANTIATE_BAL(kAmbientIblDiffuse, false, true)
PBR_INSTANTIATE_BAL(kAmbientIblDiffuse, true, false)
PBR_INSTANTIATE_BAL(kAmbientIblDiffuse, true, true)
#undef PBR_INSTANTIATE_BAL

// Development builds with PBR_BAL_PROFILE: read (and optionally clear) the balanced pass's clock sums.
hipError_t debug_bal_profile(unsigned long long* out8, bool reset) {
#if PBR_BAL_PROFILE
    constexpr size_t kWaves = 1 << 18, kBytes = kWaves * 16 * sizeof(unsigned long long);
    static unsigned long long* buf = nullptr;
    hipError_t e = hipSuccess;
    if (!buf) {
        e = hipMalloc(&buf, kBytes);
        if (e == hipSuccess) e = hipMemset(buf, 0, kBytes);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_bal_prof_buf), &buf, sizeof(buf));
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(kWaves * 16);
    if (e == hipSuccess) e = hipMemcpy(h.data(), buf, kBytes, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i) out8[i] = 0;
    for (size_t w = 0; w < kWaves; ++w)
        for (int i = 0; i < 16; ++i) out8[i] += h[w * 16 + i];
    if (e == hipSuccess && reset) e = hipMemset(buf, 0, kBytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e;
#else
    (void)out8;
    (void)reset;
    return hipErrorNotSupported;
#endif
}

#endif

// Development builds with PBR_WAVE_TIMELINE: point this translation unit's kernels at a device buffer of
// cap * kTlWords words (nullptr: off).
#if PBR_BAL_TU
hipError_t debug_wave_timeline_bal(unsigned long long* buf, long long cap) {
#else
hipError_t debug_wave_timeline_bal(unsigned long long* buf, long long cap);
hipError_t debug_wave_timeline(unsigned long long* buf, long long cap) {
#endif
#if PBR_WAVE_TIMELINE
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_wave_tl), &buf, sizeof(buf));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_wave_tl_cap), &cap, sizeof(cap));
#if !PBR_BAL_TU && PBR_SPLIT_BAL
    if (e == hipSuccess) e = debug_wave_timeline_bal(buf, cap);
#endif
    return e;
#else
    (void)buf;
    (void)cap;
    return hipErrorNotSupported;
#endif
}

// PBR_DEBUG_BOUNDS builds: point this translation unit's kernels at the device's bounds-flag buffer
// (2 * kBoundsClasses words, pbr_debug_bounds.h; one process-wide buffer per device, current device).
#if PBR_BAL_TU
hipError_t debug_bounds_publish_bal(uint32_t* buf) {
#else
hipError_t debug_bounds_publish_bal(uint32_t* buf);
hipError_t debug_bounds_publish(uint32_t* buf) {
#endif
#if PBR_DEBUG_BOUNDS
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_flags), &buf, sizeof(buf));
#if !PBR_BAL_TU && PBR_SPLIT_BAL
    if (e == hipSuccess) e = debug_bounds_publish_bal(buf);
#endif
    return e;
#else
    (void)buf;
    return hipErrorNotSupported;
#endif
}

#if !PBR_BAL_TU
__global__ void decode_unorm16_kernel(const uint16_t* __restrict__ src, float4* __restrict__ dst, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const ushort4 t = reinterpret_cast<const ushort4*>(src)[i];
        // R16G16B16A16_UNORM decode (WICTextureLoader.cpp:312-367): value / 65535
        dst[i] = make_float4((float)t.x / 65535.0f, (float)t.y / 65535.0f, (float)t.z / 65535.0f, (float)t.w / 65535.0f);
    }
}

template <int AMBIENT, bool F0_PLANE, bool APPLY_AO, bool CULL>
static hipError_t launch_variant(const LaunchArgs& a, hipStream_t stream) {
    if (a.pixels_per_thread == 2) {
        dim3 grid((a.gb.width + kTileW - 1) / kTileW, (a.gb.height + kTileH - 1) / kTileH);
        if (!CULL && a.ps.balanced != 0)
            return launch_balanced<AMBIENT, F0_PLANE, APPLY_AO>(a, grid, stream);
        if (a.lean) {  // uniform loops, no sky pass (shade_lean_kernel): one wave per workgroup
            const dim3 wgrid(grid.x, (PBR_LEAN_TILES == 2 && !CULL ? (grid.y + 1) / 2 : grid.y) * (kBlock / 64));
            if (a.ps.faithful)
                hipLaunchKernelGGL((shade_lean_kernel<AMBIENT, F0_PLANE, APPLY_AO, CULL, true>), wgrid, dim3(64), 0,
                                   stream, a.gb, a.ps, a.lights, a.env, a.frame, a.tile_kept);
            else
                hipLaunchKernelGGL((shade_lean_kernel<AMBIENT, F0_PLANE, APPLY_AO, CULL, false>), wgrid, dim3(64), 0,
                                   stream, a.gb, a.ps, a.lights, a.env, a.frame, a.tile_kept);
        } else
            hipLaunchKernelGGL((shade_tile_kernel<AMBIENT, F0_PLANE, APPLY_AO, CULL>), grid, dim3(kBlock), 0, stream,
                               a.gb, a.ps, a.lights, a.env, a.frame, a.tile_kept, a.exact_only);
    } else {
        dim3 grid((a.gb.width + kTileW1 - 1) / kTileW1, (a.gb.height + kTileH - 1) / kTileH);
        hipLaunchKernelGGL((shade_tile1_kernel<AMBIENT, F0_PLANE, APPLY_AO, CULL>), grid, dim3(kBlock), 0, stream,
                           a.gb, a.ps, a.lights, a.env, a.frame, a.tile_kept, a.exact_only);
    }
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

std::string launched_kernel(const LaunchArgs& a) {
    if (a.gb.width <= 0 || a.gb.height <= 0) return "";
    auto b = [](bool v) { return v ? std::string("true") : std::string("false"); };
    const std::string t = std::to_string(a.ambient_mode == kAmbientIblDiffuse ? 1 : 0) + ", " + b(a.f0_plane) + ", " +
                          b(a.apply_ao) + ", " + b(a.cull);
    if (a.pixels_per_thread != 2) return "shade_tile1_kernel<" + t + ">";
    if (!a.cull && a.ps.balanced != 0) return "shade_tile_kernel<" + t + ", " + std::to_string(a.ps.balanced) + ">";
    if (a.lean) return "shade_lean_kernel<" + t + ", " + b(a.ps.faithful != 0) + ">";
    return "shade_tile_kernel<" + t + ", 0>";
}

int64_t shade_tile_count(int width, int height, int pixels_per_thread) {
    const int tw = pixels_per_thread == 2 ? kTileW : kTileW1;
    return (int64_t)((width + tw - 1) / tw) * ((height + kTileH - 1) / kTileH);
}

int shade_stat_slots_per_tile(int pixels_per_thread) { return pixels_per_thread == 2 ? kBlock / 64 : 1; }

hipError_t launch_decode_unorm16(const uint16_t* src, float4* dst, int n_texels, hipStream_t stream) {
    if (n_texels <= 0) return hipSuccess;
    hipLaunchKernelGGL(decode_unorm16_kernel, dim3((n_texels + 255) / 256), dim3(256), 0, stream, src, dst, n_texels);
    return hipGetLastError();
}

#endif  // !PBR_BAL_TU

}  // namespace pbr

// This unit's build record (pbr_build_info.h, pbr_build_info): the stamp, flavor and flags it was compiled with and
// every build switch of the kernels as the preprocessor saw it.
#include "pbr_build_info.h"
#define PBR_KERNEL_SWITCHES                                                                                   \
    PBR_BI_SWITCH(PBR_X2_MIN_WAVES) ", " PBR_BI_SWITCH(PBR_LEAN_MIN_WAVES) ", "                                 \
    PBR_BI_SWITCH(PBR_LEAN_UNIFORM_MIN_WAVES) ", " PBR_BI_SWITCH(PBR_BAL_PROFILE) ", "                          \
    PBR_BI_SWITCH(PBR_WAVE_TIMELINE) ", " PBR_BI_SWITCH(PBR_DEBUG_BOUNDS) ", " PBR_BI_SWITCH(PBR_SPLIT_BAL) ", " \
    PBR_BI_SWITCH(PBR_POW5_LDS) ", " PBR_BI_SWITCH(PBR_POW5_GLIBC_FROM) ", "                                     \
    PBR_BI_SWITCH(PBR_POW5_FAST3_GLIBC_FROM) ", " PBR_BI_SWITCH(PBR_FAITHFUL_GAMMA_LO) ", "                      \
    PBR_BI_SWITCH(PBR_ATAN2F_KMAX) ", " PBR_BI_SWITCH(PBR_CENSUS) ", " PBR_BI_SWITCH(PBR_LEAN_TILES) ", "    \
    PBR_BI_SWITCH(PBR_BAL_WAVES)
#if PBR_BAL_TU
extern "C" __attribute__((used, visibility("default"))) const char pbr_unit_info_shade_kernels_bal[] =
    PBR_UNIT_INFO("shade_kernels_bal", PBR_KERNEL_SWITCHES);
#else
extern "C" __attribute__((used, visibility("default"))) const char pbr_unit_info_shade_kernels[] =
    PBR_UNIT_INFO("shade_kernels", PBR_KERNEL_SWITCHES);
#endif
