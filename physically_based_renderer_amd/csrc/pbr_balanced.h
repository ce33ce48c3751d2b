// pbr_balanced.h -- back-face-rejected, wave-balanced point-light lists for the pair kernel.
//
// Why: BRDFCookTorrance returns (kD albedo / PI + spec) * radiance * max(N.L, 0) (LightingUtil.hlsl:85-104),
// and with N.L <= 0 every factor of it is finite inside the fast-path window, so the term is +-0: adding it
// to the running sum (which starts at +0 and is never -0) is the identity. In the BASELINE scenes about half
// of all (pixel, light) terms are such zeros (normals uniform on the sphere), yet the uniform light loop
// evaluates every one of them. A per-lane skip does not pay in SIMD: the number of lights that reach a pixel
// ranges over 0..L within a wave (config 3: mean 32 of 64, max over a wave's 128 pixels ~64), so the wave
// would still run L iterations. Instead each wave
//   1. (pass 1) tests every (pixel, light) pair with a cheap conservative back-face test (below) and keeps a
//      64-bit mask of the lights that may reach each of its 128 pixels;
//   2. ranks its pixels by live-light count (LDS counting sort) and re-pairs them across lanes, the k-th
//      smallest count with the k-th largest, moving each pixel's loop invariants through LDS;
//   3. (pass 2) lets every lane walk its two pixels' live lights one after the other, TWO lights of the
//      current pixel per iteration in packed fp32 (the pixel's invariants are splat operands, the two lights'
//      records per element) -- the cycles of one packed pair-loop iteration for two items, ~L/4 iterations
//      per pixel instead of L/2 pair iterations, and all lanes finish together (a scalar one-item loop costs
//      the same VALU cycles per item as a packed two-item one on gfx950, measured: 1.32 vs 1.14 ms);
//   4. hands each pixel's sum back to the lane that owns it (LDS), which finishes the pixel as before.
// Every pixel's live lights are summed by one lane, in two interleaved partial sums (even and odd live
// lights) added at the end: a different association than the reference's, inside the faithful bound
// (non-negative terms).
//
// The back-face test (pass 1) for light j at p_j and pixel P (l = p_j - P, the reference's L before it is
// normalised), three FMAs per pixel and light (c |N|_1 B - N.P is formed once per pixel, with one rounding):
//   skip  <=>  t1 = N.p_j - N.P + c |N|_1 B < 0     (c = 2^-18 = 64u, u = 2^-24; B = max_j B_j >= B_j: a larger
//                                                   margin only skips less, and the proof below holds for it)
// B_j = B0_j + (|p_j|_1 + Pmax) / 8 (times 1 + 2^-20), where B0_j >= |l| for every pixel of the wave (the
// L1 distance from the light to the centre of the wave's position box plus the box's L1 half-extent, with
// margins for their roundings) and Pmax is the wave's largest |P|_1; computed once per wave, one lane per
// light. The FMA chain's error is <= 7u (c |N|_1 B_j + |N|_inf (|p_j|_1 + |P|_1)), and the second term of
// B_j covers the second part (c / 8 = 8u > 7u), so t1 < 0 gives N.l < -c |N|_1 |l| (1 - 7u). That bounds the
// reference's max(dot(N, L), 0) (L = l / length(l), HLSL dot; its rounding error is <= ~9u |N|_1) to 0.
// With N.L = 0 the reference's term is +-0 whatever H is: where V + L = 0 its H = normalize(V + L) is NaN, but
// max(dot(N, H), 0) and saturate(dot(H, V)) map NaN to 0 (IEEE maxNum, LightingUtil.hlsl:55, 45), so NDF and
// F stay finite and G = 0. The pixel on the light (l = 0: L = 0 / 0 = NaN) is the same case. Every other
// factor is finite for a pixel and light inside the fast-path window (the lean-wave bounds of brdf_x2: den in
// [2^-37, PI], F0 window; attenuation <= 1e4). So every skipped term is +-0 in the reference and needs no
// window test; live items run the |V + L| >= 2^-30 test in pass 2, and their distance window (a light closer than
// 0.01, 2^-20 in exact mode) is decided in pass 1 (balanced_pass1: near_a / near_b), so either sends the pixel to the
// exact re-pass as the plain loop would, here only when the item is live. Lights whose fast-path flag is off (pbr_set_pass) make the host choose the uniform loop
// (PassArgs::balanced), which sends every pixel to the exact re-pass.
#pragma once
#include <cstdint>
#include <type_traits>

#include "pbr_device_math.h"
#include "pbr_device_math_x2.h"
#include "shade_kernels.h"

namespace pbr {

constexpr int kBalRec = 7;         // float4 per exchanged pixel record

// Per-wave LDS: the exchange region (one record per lane, then the 128 results) and the count histogram.
#ifndef PBR_BAL_PROFILE
#define PBR_BAL_PROFILE 0  // development build: per-phase shader-clock sums (pbr_debug_bal_profile)
#endif
#if PBR_BAL_PROFILE
// [0] pass 1, [1] rank + exchange, [2] pass 2, [3] hand-back, [4] waves, [5] pass-2 iterations,
// [6] whole kernel (entry to the stores), [7] entry to the light loop, [8] light loop end to the reloaded
// invariants, [9] the exact re-pass barrier; the unbalanced kernel's faithful lean waves: [11] entry to the
// light loop, [12] the light loop, [13] waves, [14] the barrier, [15] entry to after the barrier
// Each wave sums its stamps in its own LDS slots (bal_prof, lane 0) and adds them to its own slots of
// g_bal_prof_buf at the end (plain loads and stores: no contended atomics to perturb the timing).
__device__ unsigned long long* g_bal_prof_buf;  // 16 per wave, wave = block * 4 + wave in block
#define BAL_PROF_T(v) const long long v = (long long)__builtin_amdgcn_s_memtime()
#define BAL_PROF_ADD(slot_, val_) do { if ((threadIdx.x & 63) == 0) bal_prof[slot_] += (unsigned long long)(val_); } while (0)
#else
#define BAL_PROF_T(v)
#define BAL_PROF_ADD(i, x)
#endif

// The pass's point lights in LDS, structure of arrays (px, py, pz, sx, sy, sz): pass 1 reads four lights'
// coordinates with one broadcast ds_read_b128 per array, pass 2's two elements read straight into a register
// pair. Entries [n, kBalLdsStride) have strength 0: pass 1 may test a padded light (position 0; its bit is masked
// off) and entry kBalMaxLights is the sentinel of pass 2 (an iteration's second element when one light is left, both
// elements of a lane with none): strength 0, so its term is (finite) * 0 = +-0, at the position kBalSentinelPos = 2^24
// on each axis, more than 2.7e7 units from any pixel of the fast window (|P| <= 2^20 per component; the distance, its
// square and the attenuation stay inside the fast division / sqrt windows), so its window test (|V + L| >= 2^-30;
// it is never a live light of pass 1's distance window) passes unless V is within ~2^-30 of the direction away from that point: a sentinel item no longer
// sends a live pixel to the exact re-pass (at position 0 it did for every pixel within 0.01 of the origin).
constexpr int kBalLdsStride = kBalMaxLights + 4;  // 68 floats: every array 16-byte aligned
constexpr float kBalSentinelPos = 0x1p24f;
// `strength_scale`: 4 for the exact balanced kernel, whose items take 4x the radiance (brdf_x2's QUARTER form; the host
// keeps every point strength within 2^50 for it, so the product cannot overflow), 1 otherwise. NT: the
// workgroup's work-items (64 in one-wave workgroups: two rounds for the 68 entries).
template <int NT = 256>
__device__ __forceinline__ void stage_balanced_lights(const float4* __restrict__ lights, int b0, int b1,
                                                      float* lds_lights, float strength_scale = 1.0f) {
    for (int t = (int)threadIdx.x; t < kBalLdsStride; t += NT) {
        float4 p = make_float4(0.0f, 0.0f, 0.0f, 0.0f), st = p;
        if (t < b1 - b0) {
            p = lights[3 * (b0 + t) + 2];
            st = lights[3 * (b0 + t)];
        } else if (t == kBalMaxLights) {
            p = make_float4(kBalSentinelPos, kBalSentinelPos, kBalSentinelPos, 0.0f);
        }
        lds_lights[0 * kBalLdsStride + t] = p.x;
        lds_lights[1 * kBalLdsStride + t] = p.y;
        lds_lights[2 * kBalLdsStride + t] = p.z;
        lds_lights[3 * kBalLdsStride + t] = st.x * strength_scale;
        lds_lights[4 * kBalLdsStride + t] = st.y * strength_scale;
        lds_lights[5 * kBalLdsStride + t] = st.z * strength_scale;
    }
}

constexpr int kBalRecX = 6;        // float4 per exchanged pixel record, exact passes

struct BalancedWaveLds {
    float4 rec[64 * kBalRec];  // 7 KiB: the exchanged records; then each evaluating lane's two results (float4 0, 1)
    union {
        int hist[64];          // ranking
        int2 rank[64];         // by owner lane: the ranks of its two pixels (pass 2 -> hand-back)
    };
};

// The per-pixel loop invariants of the faithful scaled lean loop (the scalar view of PixelInvariants2 after
// faithful_scale plus Faithful2), the pixel's live-light mask and where it came from.
struct ItemPixel {
    f3 pos, n, v, f0, omf0, mab;
    float a2m1, k, omk, nv, a2gv;
    uint32_t live0, live1;  // lights [0, 32) and [32, 64) of the pass: bit j % 32
    int origin;             // owner lane * 2 + element
};

__device__ __forceinline__ ItemPixel item_pixel(const PixelInvariants2& q, const Faithful2& fi, const f3x2& pos, int e,
                                                uint32_t live0, uint32_t live1, int origin) {
    ItemPixel r;
    r.pos = lane(pos, e);
    r.n = lane(q.n, e);
    r.v = lane(q.v, e);
    r.f0 = lane(q.f0, e);
    r.omf0 = lane(q.one_minus_f0, e);
    r.mab = lane(fi.mabpi, e);
    r.a2m1 = e ? q.a_sqr_minus_1.y : q.a_sqr_minus_1.x;
    r.k = e ? q.k.y : q.k.x;
    r.omk = e ? q.one_minus_k.y : q.one_minus_k.x;
    r.nv = e ? q.four_n_dot_v.y : q.four_n_dot_v.x;
    r.a2gv = e ? fi.a2gv.y : fi.a2gv.x;
    r.live0 = live0;
    r.live1 = live1;
    r.origin = origin;
    return r;
}

// A record's dwords go to LDS two at a time from wherever they sit in registers (ds_write2_b32): as float4 stores the
// compiler first assembled each quad in four consecutive VGPRs -- ~20 v_mov per record, four records per lane (rank
// phase). `dw` counts dwords from `dst`. Inline asm with a memory clobber: the LDS instructions of one wave execute in
// order, so the loads after the wave_lds_sync that follows see the data.
template <int DW>
__device__ __forceinline__ void lds_write2(uint32_t addr, float a, float b) {
    static_assert(DW >= 0 && DW + 1 <= 255, "ds_write2_b32 offsets are 8-bit dword counts");
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(addr), "v"(a), "v"(b), "i"(DW), "i"(DW + 1)
                 : "memory");
}
template <int DW>
__device__ __forceinline__ void lds_write1(uint32_t addr, float a) {
    asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(addr), "v"(a), "i"(4 * DW) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    typedef __attribute__((address_space(3))) const char lds_char;
    return (uint32_t)(uintptr_t)(const lds_char*)p;
}

// The faithful record: the float4 layout load_item reads (dwords 0-25; 26, 27 unused).
__device__ __forceinline__ void store_item(float4* dst, const ItemPixel& p) {
    const uint32_t a = lds_addr(dst);
    lds_write2<0>(a, p.pos.x, p.pos.y);
    lds_write2<2>(a, p.pos.z, p.n.x);
    lds_write2<4>(a, p.n.y, p.n.z);
    lds_write2<6>(a, p.v.x, p.v.y);
    lds_write2<8>(a, p.v.z, p.f0.x);
    lds_write2<10>(a, p.f0.y, p.f0.z);
    lds_write2<12>(a, p.omf0.x, p.omf0.y);
    lds_write2<14>(a, p.omf0.z, p.mab.x);
    lds_write2<16>(a, p.mab.y, p.mab.z);
    lds_write2<18>(a, p.a2m1, p.k);
    lds_write2<20>(a, p.omk, p.nv);
    lds_write2<22>(a, p.a2gv, __uint_as_float(p.live0));
    lds_write2<24>(a, __uint_as_float(p.live1), __int_as_float(p.origin));
}
__device__ __forceinline__ ItemPixel load_item(const float4* src) {
    const float4 a = src[0], b = src[1], c = src[2], d = src[3], e = src[4], f = src[5], g = src[6];
    ItemPixel p;
    p.pos = mk3(a.x, a.y, a.z);
    p.n = mk3(a.w, b.x, b.y);
    p.v = mk3(b.z, b.w, c.x);
    p.f0 = mk3(c.y, c.z, c.w);
    p.omf0 = mk3(d.x, d.y, d.z);
    p.mab = mk3(d.w, e.x, e.y);
    p.a2m1 = e.z;
    p.k = e.w;
    p.omk = f.x;
    p.nv = f.y;
    p.a2gv = f.z;
    p.live0 = __float_as_uint(f.w);
    p.live1 = __float_as_uint(g.x);
    p.origin = __float_as_int(g.y);
    return p;
}

// The exact (default-mode) record: the lean-loop invariants of make_invariants in brdf_x2's QUARTER form (N / 4, k / 4,
// 16 N.V: exact scalings), less the three that are one subtraction from another field (1 - F0, a^2 - 1, 1 - k:
// re-derived by load_item_x with the same operation on the unscaled value, so bit for bit the same values). The pixel's sum so far (its directional lights), from which the
// evaluating lane continues in the reference's order, travels separately (BalancedWaveLds::start): written by
// the owner before the exchange, it is not held in registers through it.
struct ItemPixelX {
    f3 pos, n, v, albedo, f0, omf0;
    float omm, a_sqr, a2m1, k, omk, ggx_v, nv4;
    uint32_t live0, live1;
    int origin;
};

__device__ __forceinline__ ItemPixelX item_pixel_x(const PixelInvariants2& q, const f3x2& pos, int e, uint32_t live0,
                                                   uint32_t live1, int origin) {
    ItemPixelX r;
    r.pos = lane(pos, e);
    const f3 n = lane(q.n, e);
    r.n = mk3(0.25f * n.x, 0.25f * n.y, 0.25f * n.z);  // QUARTER
    r.v = lane(q.v, e);
    r.albedo = lane(q.albedo, e);
    r.f0 = lane(q.f0, e);
    r.omm = e ? q.one_minus_metal.y : q.one_minus_metal.x;
    r.a_sqr = e ? q.a_sqr.y : q.a_sqr.x;
    r.k = 0.25f * (e ? q.k.y : q.k.x);                       // QUARTER: k / 4
    r.ggx_v = e ? q.ggx_v.y : q.ggx_v.x;
    r.nv4 = 4.0f * (e ? q.four_n_dot_v.y : q.four_n_dot_v.x);  // QUARTER: 16 N.V
    r.live0 = live0;
    r.live1 = live1;
    r.origin = origin;
    return r;
}

// The exact record: the float4 layout load_item_x reads (dwords 0-22; 23 unused).
__device__ __forceinline__ void store_item(float4* dst, const ItemPixelX& p) {
    const uint32_t a = lds_addr(dst);
    lds_write2<0>(a, p.pos.x, p.pos.y);
    lds_write2<2>(a, p.pos.z, p.n.x);
    lds_write2<4>(a, p.n.y, p.n.z);
    lds_write2<6>(a, p.v.x, p.v.y);
    lds_write2<8>(a, p.v.z, p.albedo.x);
    lds_write2<10>(a, p.albedo.y, p.albedo.z);
    lds_write2<12>(a, p.f0.x, p.f0.y);
    lds_write2<14>(a, p.f0.z, p.omm);
    lds_write2<16>(a, p.a_sqr, p.k);
    lds_write2<18>(a, p.ggx_v, p.nv4);
    lds_write2<20>(a, __uint_as_float(p.live0), __uint_as_float(p.live1));
    lds_write1<22>(a, __int_as_float(p.origin));
}
__device__ __forceinline__ ItemPixelX load_item_x(const float4* src) {
    const float4 a = src[0], b = src[1], c = src[2], d = src[3], e = src[4], f = src[5];
    ItemPixelX p;
    p.pos = mk3(a.x, a.y, a.z);
    p.n = mk3(a.w, b.x, b.y);
    p.v = mk3(b.z, b.w, c.x);
    p.albedo = mk3(c.y, c.z, c.w);
    p.f0 = mk3(d.x, d.y, d.z);
    p.omm = d.w;
    p.a_sqr = e.x;
    p.k = e.y;
    p.ggx_v = e.z;
    p.nv4 = e.w;
    p.live0 = __float_as_uint(f.x);
    p.live1 = __float_as_uint(f.y);
    p.origin = __float_as_int(f.z);
    p.omf0 = mk3(1.0f - p.f0.x, 1.0f - p.f0.y, 1.0f - p.f0.z);  // make_invariants' operations
    p.a2m1 = 16.0f * (p.a_sqr - 1.0f);                           // QUARTER: 16 (a^2 - 1)
    p.omk = 1.0f - 4.0f * p.k;                                   // 1 - k (4 (k / 4) is k exactly)
    return p;
}
template <bool EXACT>
__device__ __forceinline__ auto load_item_any(const float4* src) {
    if constexpr (EXACT)
        return load_item_x(src);
    else
        return load_item(src);
}

// LDS traffic of one wave between its own lanes: the hardware executes a wave's LDS instructions in order;
// the fences keep the compiler from moving them across this point.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Pass 1 runs in fast-window waves only (lean and faithful or exact lean: every position |x| <= 2^20, every light inside
// its window), so every value it reduces is finite: the float-unit reductions (wave_minmax_finite).
// FINITE: the faithful kernel's pass 1. The exact balanced kernel keeps the order-key reductions (wave_min_dpp): with
// the float-unit ones its SGPR spills to VGPR lanes grew (295 -> 361 lane moves in the kernel) and config 3 exact
// measured ~1% slower.
template <bool FINITE>
__device__ __forceinline__ float bal_wave_min(float v) {
    if constexpr (FINITE) return wave_min_finite(v);
    else return wave_min_dpp(v);
}
template <bool FINITE>
__device__ __forceinline__ float bal_wave_max(float v) {
    if constexpr (FINITE) return wave_max_finite(v);
    else return wave_max_dpp(v);
}
template <bool FINITE>
__device__ __forceinline__ float bal_fmin(float a, float b) {
    if constexpr (FINITE) return fmin_finite(a, b);
    else return fminf(a, b);
}
template <bool FINITE>
__device__ __forceinline__ float bal_fmax(float a, float b) {
    if constexpr (FINITE) return fmax_finite(a, b);
    else return fmaxf(a, b);
}

// Pass 1 for the pair and four lights j..j+3 (coordinates x, y, z: one float4 per axis, light j + i in element i):
// shift the lights' SKIP bits for each pixel (the sign of t1, see the header comment) into `ma` / `mb`, light j + 3
// first, so that light j ends lowest. kb = c |N|_1 B - N.P per pixel, with the wave's bound B = max_j B_j (any B >= B_j
// keeps the skip proof: the margin term only grows), so the test is three FMAs per pixel and light:
// t1 = N.x l.x + (N.y l.y + (N.z l.z + kb)). Each packed FMA takes two LIGHTS of one pixel (the light pairs are the
// quads' aligned halves, the pixel's values splat operands of the loop-invariant pixel pair): the earlier form (two
// pixels, one light splat from the quad) overwrote quads it still had to splat from, which cost ~0.9 moves per light.
__device__ __forceinline__ void push_skip_bits4(uint32_t& ma, uint32_t& mb, float4 x, float4 y, float4 z,
                                                const f3x2& n, v2 kb) {
    const v2 x01 = v2{x.x, x.y}, x23 = v2{x.z, x.w}, y01 = v2{y.x, y.y}, y23 = v2{y.z, y.w};
    const v2 z01 = v2{z.x, z.y}, z23 = v2{z.z, z.w};
    const v2 ta01 = vfma(splat(n.x.x), x01, vfma(splat(n.y.x), y01, vfma(splat(n.z.x), z01, splat(kb.x))));
    const v2 ta23 = vfma(splat(n.x.x), x23, vfma(splat(n.y.x), y23, vfma(splat(n.z.x), z23, splat(kb.x))));
    const v2 tb01 = vfma(splat(n.x.y), x01, vfma(splat(n.y.y), y01, vfma(splat(n.z.y), z01, splat(kb.y))));
    const v2 tb23 = vfma(splat(n.x.y), x23, vfma(splat(n.y.y), y23, vfma(splat(n.z.y), z23, splat(kb.y))));
    ma = __builtin_amdgcn_alignbit(ma, __float_as_uint(ta23.y), 31);  // (m << 1) | sign(t1)
    mb = __builtin_amdgcn_alignbit(mb, __float_as_uint(tb23.y), 31);
    ma = __builtin_amdgcn_alignbit(ma, __float_as_uint(ta23.x), 31);
    mb = __builtin_amdgcn_alignbit(mb, __float_as_uint(tb23.x), 31);
    ma = __builtin_amdgcn_alignbit(ma, __float_as_uint(ta01.y), 31);
    mb = __builtin_amdgcn_alignbit(mb, __float_as_uint(tb01.y), 31);
    ma = __builtin_amdgcn_alignbit(ma, __float_as_uint(ta01.x), 31);
    mb = __builtin_amdgcn_alignbit(mb, __float_as_uint(tb01.x), 31);
}

// Pass 2's light records for one iteration (element 0: light j0; element 1: light j1; index kBalMaxLights is the
// zero sentinel: position and strength 0) from the SoA staging: all twelve LDS reads issued back to back and one
// wait. Left to itself the compiler interleaved reads and waits (three or four round trips per iteration), and the
// waves run this loop nearly in step, so each round trip idled the SIMD.
__device__ __forceinline__ void read_pair_lights(const float* lds_lights, int j0, int j1, f3x2& lp, f3x2& ls) {
    typedef __attribute__((address_space(3))) const float lds_float;
    j0 = PBR_BOUNDS(j0, kBalMaxLights + 1, kBoundsLds);
    j1 = PBR_BOUNDS(j1, kBalMaxLights + 1, kBoundsLds);
    const uint32_t base = (uint32_t)(uintptr_t)(const lds_float*)lds_lights;
    const uint32_t a0 = base + 4u * (uint32_t)j0, a1 = base + 4u * (uint32_t)j1;
    float x0, x1, y0, y1, z0, z1, r0, r1, g0, g1, u0, u1;
    static_assert(kBalLdsStride * 4 == 272, "offsets below");
    asm volatile(
        "ds_read_b32 %0, %12\n\t"
        "ds_read_b32 %1, %13\n\t"
        "ds_read_b32 %2, %12 offset:272\n\t"
        "ds_read_b32 %3, %13 offset:272\n\t"
        "ds_read_b32 %4, %12 offset:544\n\t"
        "ds_read_b32 %5, %13 offset:544\n\t"
        "ds_read_b32 %6, %12 offset:816\n\t"
        "ds_read_b32 %7, %13 offset:816\n\t"
        "ds_read_b32 %8, %12 offset:1088\n\t"
        "ds_read_b32 %9, %13 offset:1088\n\t"
        "ds_read_b32 %10, %12 offset:1360\n\t"
        "ds_read_b32 %11, %13 offset:1360\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1), "=&v"(y0), "=&v"(y1), "=&v"(z0), "=&v"(z1), "=&v"(r0), "=&v"(r1), "=&v"(g0),
          "=&v"(g1), "=&v"(u0), "=&v"(u1)
        : "v"(a0), "v"(a1)
        : "memory");
    lp = f3x2{v2{x0, x1}, v2{y0, y1}, v2{z0, z1}};
    ls = f3x2{v2{r0, r1}, v2{g0, g1}, v2{u0, u1}};
}

// ---- pass 2: two (pixel, light) items of the faithful scaled lean loop, packed ---------------------------
// ComputePointLight (LightingUtil.hlsl:124-142) + BRDFCookTorrance for ONE pixel (q, splat into both elements)
// and TWO lights (element e: position lp.*[e], strength ls.*[e]), added into `sum`: the operations of
// point_or_spot_faithful_x2<false, true, true> / brdf_faithful_x2<true, true> element for element (same
// roundings, same window tests into `ok`), but for the Fresnel x^5 (pow5_fast3, three products) and the range cut of
// LightingUtil.hlsl:131: pass 1 removed every item whose light is beyond the range of its pixel (balanced_pass1), so
// each item here is within range and the 0/1 factor in_range01 would be exactly 1 (the sentinel's zero strength
// still zeroes its term).
// The two rare cases of an item share one test: |V + L| (the length normalize(V + L) divides by) below kBalNearVL.
// Unit V and L give H.V = |V + L| / 2 (with |V|, |L| = 1 within a few 2^-24, H.V >= |V + L| / 2 - 2^-21 / |V + L| after
// the roundings), so |V + L| >= 1/16 gives H.V > 0.0312 and x = 1 - H.V < 0.9688: below pow5_fast3's glibc band
// (x > 0.97), and far above normalize_x2's window (|V + L| >= 2^-30). Only when a live lane's item falls below 1/16 (L
// within ~3.6 degrees of -V: rare, as the glibc band is) does the wave run the window test and the band patch, as a
// uniform branch: 2 compares per iteration instead of 4.
constexpr float kBalNearVL = 0.0625f;
__device__ __forceinline__ void faithful_point_items2(const ItemPixel& q, const f3x2& lp, const f3x2& ls, m2& ok,
                                                      f3x2& sum, uint64_t live) {
    f3x2 l = f3x2{lp.x - q.pos.x, lp.y - q.pos.y, lp.z - q.pos.z};
    const v2 dist = sqrt_nr(dot3(l, l));  // >= 0.01 for a live item of a pixel pass 1 did not redo
    const Recip2 rdist = recip_nr(dist);
    l = f3x2{div_nr(l.x, rdist), div_nr(l.y, rdist), div_nr(l.z, rdist)};
    const f3x2 vl = f3x2{q.v.x + l.x, q.v.y + l.y, q.v.z + l.z};
    const v2 svl = sqrt_nr(dot3(vl, vl));  // normalize_x2's operations, its window test below
    const Recip2 rvl = recip_nr(svl);
    const f3x2 h = f3x2{div_nr(vl.x, rvl), div_nr(vl.y, rvl), div_nr(vl.z, rvl)};
    const v2 att = rdist.r * rdist.r;
    const f3x2 n = splat3(q.n.x, q.n.y, q.n.z);
    const v2 n_dot_h = dot3_sat(n, h);
    const v2 inner = ((n_dot_h * n_dot_h) * q.a2m1 + 1.0f);
    const v2 den = inner * inner;
    const v2 n_dot_l = dot3_sat(n, l);
    const v2 r = rcp_hw((den * vfma(n_dot_l, splat(q.omk), splat(q.k))) * vfma(splat(q.nv), n_dot_l, splat(0.001f)));
    const v2 x = 1.0f - dot3_sat(h, splat3(q.v.x, q.v.y, q.v.z));
    const v2 x2 = x * x;
    const v2 x4 = x2 * x2;
    v2 p = x4 * x;  // pow5_fast3's products
    if (__builtin_expect(((lanes(svl.x < kBalNearVL) | lanes(svl.y < kBalNearVL)) & live) != 0, 0)) {
        ok &= ge(svl, 0x1p-30f);  // normalize_x2's window
        if (x.x > PBR_POW5_FAST3_GLIBC_FROM && on(live)) p.x = pow5_glibc(x.x);  // pow5_fast3's band
        if (x.y > PBR_POW5_FAST3_GLIBC_FROM && on(live)) p.y = pow5_glibc(x.y);
    }
    const f3x2 f = f3x2{q.f0.x + q.omf0.x * p, q.f0.y + q.omf0.y * p, q.f0.z + q.omf0.z * p};
    const v2 kr = (q.a2gv * n_dot_l) * r;
    const v2 w = att * n_dot_l;
    sum.x = vfma(vfma(kr, f.x, vfma(-f.x, splat(q.mab.x), splat(q.mab.x))), ls.x * w, sum.x);
    sum.y = vfma(vfma(kr, f.y, vfma(-f.y, splat(q.mab.y), splat(q.mab.y))), ls.y * w, sum.y);
    sum.z = vfma(vfma(kr, f.z, vfma(-f.z, splat(q.mab.z), splat(q.mab.z))), ls.z * w, sum.z);
}

// The same two items on the exact lean loop: point_or_spot_x2<false, true> (pbr_device_math_x2.h) for one pixel
// and two lights, element for element the same operations (the pixel's invariants splat into both elements), so
// each element's term carries the bits of the uniform loop's term for that (pixel, light), less the range factor,
// which is exactly 1 for every item pass 1 keeps (faithful_point_items2): the bits are unchanged.
__device__ __forceinline__ f3x2 exact_point_items2(const ItemPixelX& p, const f3x2& lp, const f3x2& ls, m2& ok,
                                                   uint64_t live) {
    PixelInvariants2 q;
    q.n = splat3(p.n.x, p.n.y, p.n.z);
    q.v = splat3(p.v.x, p.v.y, p.v.z);
    q.albedo = splat3(p.albedo.x, p.albedo.y, p.albedo.z);
    q.f0 = splat3(p.f0.x, p.f0.y, p.f0.z);
    q.one_minus_f0 = splat3(p.omf0.x, p.omf0.y, p.omf0.z);
    q.one_minus_metal = splat(p.omm);
    q.a_sqr = splat(p.a_sqr);
    q.a_sqr_minus_1 = splat(p.a2m1);
    q.k = splat(p.k);
    q.one_minus_k = splat(p.omk);
    q.ggx_v = splat(p.ggx_v);
    q.four_n_dot_v = splat(p.nv4);
    q.f0_nonzero = m2{~0ull, ~0ull};  // not read by the lean BRDF
    f3x2 l = f3x2{lp.x - p.pos.x, lp.y - p.pos.y, lp.z - p.pos.z};
    const v2 dist = sqrt_nr(dot3(l, l));  // >= 2^-20 (kBalDistLoExact) unless pass 1 redoes the pixel
    const Recip2 rdist = recip_nr(dist);
    l = f3x2{div_nr(l.x, rdist), div_nr(l.y, rdist), div_nr(l.z, rdist)};
    const f3x2 h = normalize_x2(add3(q.v, l), ok);
    const v2 dsat = max_dsat(dist);
    const v2 att = recip_nr(dsat * dsat).r;
    return brdf_x2<true, true>(q, f3x2{ls.x * att, ls.y * att, ls.z * att}, l, h, ok, live);  // ls: 4x strengths
}

// The live-light masks of the pair's pixels (pass 1), light j at bit j % 32 of word j / 32.
struct BalMasks {
    uint32_t a0, a1, c0, c1;  // pixel a: lights [0, 32), [32, 64); pixel b: the same
    bool near_a, near_b;      // the pixel has a live light closer than the distance window (pass 1): redo it
};

// The distance windows of the two item forms (the lean loops' `ge(dist, lo)` of point_or_spot_faithful_x2 and
// point_or_spot_x2), decided in pass 1 instead of per item.
constexpr float kBalDistLoFaithful = 0.01f;
constexpr float kBalDistLoExact = 0x1p-20f;

// The reference's range cut (LightingUtil.hlsl:129-131: d = length(lightVec); if (d > 100) return 0) as pass 1 applies it
// to a light whose range boundary crosses the wave's box: d = RN(sqrt(x)) with x = dot(l, l) in HLSL order (the kernel's
// sqrt_nr is the correctly rounded sqrt in the window), and RN(sqrt(x)) <= 100 <=> sqrt(x) <= 100 + 2^-18 (the midpoint
// to the next float, 2^-17 above 100, rounds to the even 100) <=> x <= (100 + 2^-18)^2 = 10000 + 7.6e-4, below the next
// float after 10000 (2^-10 above it): d > 100 <=> x > 10000, decided bit for bit as the reference decides it.
__device__ __forceinline__ m2 beyond_range(const f3x2& pos, float lx, float ly, float lz) {
    const f3x2 l = f3x2{splat(lx) - pos.x, splat(ly) - pos.y, splat(lz) - pos.z};
    const v2 x = dot3(l, l);
    return mask2(x.x > 10000.0f, x.y > 10000.0f);
}

// Pass 1 for point lights [0, nl) of the pass (staged in `lds_lights`), from the pair's raw G-buffer position
// and normal (the test is invariant under scaling N): run before the loop invariants exist, so that the two
// never hold registers at the same time. Wave-uniform control flow.
// The range cut (LightingUtil.hlsl:131) is applied here too, so pass 2 evaluates no item beyond the range and carries
// no range test: a light farther than 100 from every pixel of the wave's box is dropped for the wave (its terms are
// the +0 the reference adds); a light whose range boundary crosses the box is tested per pixel (beyond_range, the
// reference's own decision), a light within 99.9 of every corner is kept as the back-face test says.
// The distance window of pass 2's items (dist >= dist_lo, kBalDistLo*) is decided here as well: a light whose box
// distance proves it (the nearest box point at least 1.02 dist_lo away: every pixel's dist >= dist_lo after the few
// roundings) needs no test; for another (rare) light each pixel whose live mask holds it runs the item's own test --
// the same dist from the same operations -- and a pixel that fails is redone on the exact path (near_a / near_b), as
// a failed window test in pass 2 would have redone it.
template <bool EXACT>
__device__ __forceinline__ BalMasks balanced_pass1(const f3x2& pos, const f3x2& n, bool live_a, bool live_b, int nl,
                                                   float dist_lo, BalancedWaveLds& w, const float* lds_lights,
                                                   unsigned long long* bal_prof = nullptr) {
    const int lane_id = (int)(threadIdx.x & 63);
    BAL_PROF_T(t0);
    // ---- pass 1: live masks of both pixels
    // The wave's position box (geometry pixels) -> centre c and L1 half-extent r; lane k computes light k's
    // bound B_k = (|p_k - c|_1 + r + |c|_1 2^-22) (1 + 2^-20) >= |p_k - P|_1 >= |p_k - P| for every pixel P of
    // the wave (the extra terms cover the roundings of c, r and B_k) into the wave's LDS region.
    const float big = 3.0e38f;
    const f3 pa = lane(pos, 0), pb = lane(pos, 1);
    constexpr bool F = !EXACT;
    const float mnx = bal_wave_min<F>(bal_fmin<F>(live_a ? pa.x : big, live_b ? pb.x : big));
    const float mny = bal_wave_min<F>(bal_fmin<F>(live_a ? pa.y : big, live_b ? pb.y : big));
    const float mnz = bal_wave_min<F>(bal_fmin<F>(live_a ? pa.z : big, live_b ? pb.z : big));
    const float mxx = bal_wave_max<F>(bal_fmax<F>(live_a ? pa.x : -big, live_b ? pb.x : -big));
    const float mxy = bal_wave_max<F>(bal_fmax<F>(live_a ? pa.y : -big, live_b ? pb.y : -big));
    const float mxz = bal_wave_max<F>(bal_fmax<F>(live_a ? pa.z : -big, live_b ? pb.z : -big));
    const float cx = 0.5f * mnx + 0.5f * mxx, cy = 0.5f * mny + 0.5f * mxy, cz = 0.5f * mnz + 0.5f * mxz;
    const float r = (0.5f * (mxx - mnx) + 0.5f * (mxy - mny)) + 0.5f * (mxz - mnz);
    const float slack = r + (fabsf(cx) + fabsf(cy) + fabsf(cz)) * 0x1p-22f;
    const float pmax = bal_wave_max<F>(bal_fmax<F>(live_a ? (fabsf(pa.x) + fabsf(pa.y)) + fabsf(pa.z) : 0.0f,
                                                   live_b ? (fabsf(pb.x) + fabsf(pb.y)) + fabsf(pb.z) : 0.0f));
    float bj = 0.0f;  // B_j of light j = lane (j < nl; padded lights: zero position, harmless), B = the maximum
    bool near = true, far = false;  // light j: within range of every pixel of the box / beyond range of every one
    bool close = false;             // light j may come closer than dist_lo to a pixel of the box (or is NaN)
    if (lane_id < nl) {
        const float lx = lds_lights[lane_id], ly = lds_lights[kBalLdsStride + lane_id],
                    lz = lds_lights[2 * kBalLdsStride + lane_id];
        const float b0 = ((fabsf(lx - cx) + fabsf(ly - cy)) + fabsf(lz - cz)) + slack;
        const float fr = ((fabsf(lx) + fabsf(ly)) + fabsf(lz)) + pmax;
        bj = (b0 + 0.125f * fr) * (1.0f + 0x1p-20f);
        // The box corner farthest from the light (per axis) and the box point nearest to it bound its distance to
        // every pixel of the wave. In fp32 with a few roundings (~5u) against the kernel's dist, itself within ~5u of
        // the true distance: a farthest corner <= 99.9 leaves every pixel's d < 100, a nearest point >= 100.1 every
        // d > 100. Neither holds for a NaN (then, or in between, the pixel test decides).
        const float fx = fmaxf(fabsf(lx - mnx), fabsf(lx - mxx)), fy = fmaxf(fabsf(ly - mny), fabsf(ly - mxy)),
                    fz = fmaxf(fabsf(lz - mnz), fabsf(lz - mxz));
        const float gx = fmaxf(fmaxf(mnx - lx, lx - mxx), 0.0f), gy = fmaxf(fmaxf(mny - ly, ly - mxy), 0.0f),
                    gz = fmaxf(fmaxf(mnz - lz, lz - mxz), 0.0f);
        near = (fx * fx + fy * fy) + fz * fz <= 99.9f * 99.9f;
        far = (gx * gx + gy * gy) + gz * gz >= 100.1f * 100.1f;
        close = !((gx * gx + gy * gy) + gz * gz >= (1.02f * dist_lo) * (1.02f * dist_lo));
    }
    const float bmax = bal_wave_max<F>(bj);
    const uint64_t far_m = lanes(far), cross_m = lanes(!near && !far), close_m = lanes(close);  // bit j: light j
    const v2 cn = v2{0x1p-18f * ((fabsf(n.x.x) + fabsf(n.y.x)) + fabsf(n.z.x)),
                     0x1p-18f * ((fabsf(n.x.y) + fabsf(n.y.y)) + fabsf(n.z.y))};
    const v2 nd = -vfma(n.z, pos.z, vfma(n.y, pos.y, n.x * pos.x));  // -N.P
    const v2 kb = vfma(cn, splat(bmax), nd);
    uint32_t a0 = 0, a1 = 0, c0 = 0, c1 = 0;  // skip bits; pixel a: a0 (lights 0..31), a1; pixel b: c0, c1
    // Four lights per step from uniform (broadcast) LDS reads, pushed from the highest light down so that
    // light j ends at bit j % 32 of its word. A word always runs all 32 of its lights (padded lights are zero
    // records whose bits are masked below): straight-line code, in which the compiler issues the LDS reads of
    // later steps ahead of the arithmetic of earlier ones -- the waves of a block run this phase nearly in
    // step, so a read waited on at once would idle the SIMD for its latency.
    // Two steps (eight lights) per LDS round trip: their sixteen 16-byte reads are issued back to back and
    // waited on once (inline asm; left to itself the compiler waited after every few reads).
    typedef __attribute__((address_space(3))) const float lds_float;
    const uint32_t lbase = (uint32_t)(uintptr_t)(const lds_float*)lds_lights;
    auto word = [&](int qbase, uint32_t& ma, uint32_t& mb) {  // lights [4 qbase, 4 qbase + 32)
        for (int k = 6; k >= 0; k -= 2) {  // steps k + 1 and k
            const uint32_t la = lbase + 16u * (uint32_t)(qbase + k);
            float4 x1, y1, z1, x0, y0, z0;  // step k + 1 (lights 4(q + k) + 4..7), step k (+ 0..3)
            asm volatile(
                "ds_read_b128 %0, %6 offset:16\n\t"
                "ds_read_b128 %1, %6 offset:288\n\t"
                "ds_read_b128 %2, %6 offset:560\n\t"
                "ds_read_b128 %3, %6\n\t"
                "ds_read_b128 %4, %6 offset:272\n\t"
                "ds_read_b128 %5, %6 offset:544\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(x1), "=&v"(y1), "=&v"(z1), "=&v"(x0), "=&v"(y0), "=&v"(z0)
                : "v"(la)
                : "memory");
            push_skip_bits4(ma, mb, x1, y1, z1, n, kb);
            push_skip_bits4(ma, mb, x0, y0, z0, n, kb);
        }
    };
    const int n0 = nl < 32 ? nl : 32;
    if (nl > 32) word(8, a1, c1);
    word(0, a0, c0);
    // Live masks (light j at bit j % 32 of its word); bits above a word's light count are not lights, nor are the
    // lights beyond range of the whole box (scalar masks: no VALU).
    const int n1 = nl - n0;
    const uint32_t k0 = (n0 == 32 ? ~0u : (1u << n0) - 1u) & ~(uint32_t)far_m,
                   k1 = (n1 == 32 ? ~0u : (1u << n1) - 1u) & ~(uint32_t)(far_m >> 32);
    a0 = live_a ? ~a0 & k0 : 0u;
    c0 = live_b ? ~c0 & k0 : 0u;
    a1 = live_a ? ~a1 & k1 : 0u;
    c1 = live_b ? ~c1 & k1 : 0u;
    // Lights whose range boundary crosses the box: the reference's decision per pixel (rare: none in the BASELINE
    // scenes, whose lights are within range of every pixel).
    for (uint64_t cm = cross_m; cm != 0; cm &= cm - 1) {  // uniform
        const int j = __builtin_ctzll(cm);
        const m2 out = beyond_range(pos, lds_lights[j], lds_lights[kBalLdsStride + j], lds_lights[2 * kBalLdsStride + j]);
        const uint32_t bit = 1u << (j & 31);
        const uint32_t oa = on(out.x) ? bit : 0u, ob = on(out.y) ? bit : 0u;
        if (j < 32) {
            a0 &= ~oa;
            c0 &= ~ob;
        } else {
            a1 &= ~oa;
            c1 &= ~ob;
        }
    }
    // Lights that may come closer than the distance window: the item's window test, per pixel (rare).
    bool near_a = false, near_b = false;
    for (uint64_t cm = close_m; cm != 0; cm &= cm - 1) {  // uniform
        const int j = __builtin_ctzll(cm);
        const f3x2 l = f3x2{splat(lds_lights[j]) - pos.x, splat(lds_lights[kBalLdsStride + j]) - pos.y,
                            splat(lds_lights[2 * kBalLdsStride + j]) - pos.z};
        const m2 ok = ge(sqrt_nr(dot3(l, l)), dist_lo);
        const uint32_t bit = 1u << (j & 31);
        near_a = near_a || (((j < 32 ? a0 : a1) & bit) != 0 && !on(ok.x));
        near_b = near_b || (((j < 32 ? c0 : c1) & bit) != 0 && !on(ok.y));
    }

    BAL_PROF_T(t1);
    BAL_PROF_ADD(0, t1 - t0);
    return BalMasks{a0, a1, c0, c1, near_a, near_b};
}

// The wave's live (pixel, light) items -- the popcounts of its pixels' live masks, summed over the wave: the
// point-light terms pass 2 evaluates (statistics: pbr_pass_stats::light_terms). Wave-uniform result.
__device__ __forceinline__ int wave_live_items(const BalMasks& bm) {
    return wave_sum_dpp((__popc(bm.a0) + __popc(bm.a1)) + (__popc(bm.c0) + __popc(bm.c1)));
}


// The whole balanced pass over the point lights of an untiled lean wave (at most kBalMaxLights). `live_a` /
// `live_b` say which of the pair's pixels take part (geometry); `lds_lights`: the pass's point lights staged by
// the block (stage_balanced_lights); `bm`: their live masks from balanced_pass1. ORs the pixels that left the
// fast-path window for a live item into `redo`. Wave-uniform control flow; no block barrier.
// EXACT (the default mode's lean loop, bit-identical to the uniform loop): q is unscaled, `sum` holds the pair's
// directional-light sums on entry; each pixel's sum continues from it through its live lights in increasing
// light order (element 0 of an iteration is the smaller light; the skipped terms are the +-0 the reference adds),
// and `sum` is replaced by the result. Faithful: q / fi scaled, the point-light sums are added into `sum`.
template <bool EXACT>
__device__ __forceinline__ void lighting_balanced_points(const PixelInvariants2& q, const Faithful2& fi,
                                                         const f3x2& pos, bool live_a, bool live_b, BalMasks bm,
                                                         BalancedWaveLds& w, const float* lds_lights, f3x2& sum,
                                                         m2& redo, unsigned long long* bal_prof = nullptr) {
    const int lane_id = (int)(threadIdx.x & 63);
    const uint32_t a0 = bm.a0, a1 = bm.a1, c0 = bm.c0, c1 = bm.c1;
    redo |= mask2(bm.near_a, bm.near_b);  // pass 1's distance window (the items carry no test)
    constexpr int R = EXACT ? kBalRecX : kBalRec;  // record stride (float4)
    BAL_PROF_T(t1);
    PBR_PHASE("rank");

    // ---- rank the wave's 128 pixels by live count (counting sort; ties in LDS-atomic order, which only
    // decides which lane evaluates a pixel, never how)
    const int cnt_a = __popc(a0) + __popc(a1), cnt_b = __popc(c0) + __popc(c1);
    w.hist[lane_id] = 0;
    wave_lds_sync();
    const int bin_a = cnt_a < 63 ? cnt_a : 63, bin_b = cnt_b < 63 ? cnt_b : 63;
    const int pos_a = atomicAdd(&w.hist[bin_a], 1);
    const int pos_b = atomicAdd(&w.hist[bin_b], 1);
    wave_lds_sync();
    const int h = w.hist[lane_id];
    const int incl = wave_scan_add_dpp(h);
    wave_lds_sync();
    w.hist[lane_id] = incl - h;  // exclusive prefix: first rank of each bin
    wave_lds_sync();
    const int rank_a = w.hist[bin_a] + pos_a, rank_b = w.hist[bin_b] + pos_b;
    wave_lds_sync();
    w.rank[lane_id] = make_int2(rank_a, rank_b);  // read back at the hand-back (nothing of it lives through pass 2)
    // rank r < 64 -> lane r, first pixel; r >= 64 -> lane 127 - r, second pixel.
    using Item = std::conditional_t<EXACT, ItemPixelX, ItemPixel>;
    Item ia, ib;
    if constexpr (EXACT) {
        ia = item_pixel_x(q, pos, 0, a0, a1, 2 * lane_id);
        ib = item_pixel_x(q, pos, 1, c0, c1, 2 * lane_id + 1);
    } else {
        ia = item_pixel(q, fi, pos, 0, a0, a1, 2 * lane_id);
        ib = item_pixel(q, fi, pos, 1, c0, c1, 2 * lane_id + 1);
    }
    // Phase 0: the small-count pixels.
    if (rank_a < 64) store_item(&w.rec[R * rank_a], ia);
    if (rank_b < 64) store_item(&w.rec[R * rank_b], ib);
    wave_lds_sync();
    Item cur = load_item_any<EXACT>(&w.rec[R * lane_id]);
    wave_lds_sync();
    // Phase 1: the large-count pixels stay in LDS; a lane reads its second pixel when it switches.
    if (rank_a >= 64) store_item(&w.rec[R * (127 - rank_a)], ia);
    if (rank_b >= 64) store_item(&w.rec[R * (127 - rank_b)], ib);
    wave_lds_sync();

    BAL_PROF_T(t2);
    PBR_PHASE("pass2");
    // ---- pass 2
    // Every lane runs every iteration (no divergent body): a lane with no live light left takes the zero sentinel
    // (index kBalMaxLights: position and strength 0) for both elements, whose terms its dead accumulator absorbs.
    // Lane state that is uniform in kind lives in scalar lane masks: `fail` (the lane's current pixel left the fast
    // window for a live item; window tests are ballots, so only the bits of lanes with live items are ORed in),
    // `second` (the lane is on its second pixel). Faithful: two interleaved partial sums (acc); exact: one running
    // sum per pixel (accx) in light order.
    f3x2 acc = splat3(0.0f, 0.0f, 0.0f);
    f3 accx = mk3(0.0f, 0.0f, 0.0f);
    uint64_t fail = 0, second = 0;
    uint64_t m = ((uint64_t)cur.live1 << 32) | cur.live0;
    // A finished pixel's result (its three sums and whether it stayed inside the fast-path window) goes to LDS at
    // once, so that nothing of it stays in registers: into the evaluating lane's own record slot, float4 0 for its
    // first pixel and 1 for its second -- the slot held the lane's second record, which the lane has read before it
    // writes there (a wave's LDS operations execute in order); the owner finds it from the pixel's rank.
    auto result = [&]() {  // divergent: the lanes whose current pixel is done
        const f3 r = EXACT ? accx : mk3(acc.x.x + acc.x.y, acc.y.x + acc.y.y, acc.z.x + acc.z.y);
        return make_float4(r.x, r.y, r.z, on(fail) ? 0.0f : 1.0f);
    };
    // Two dwords at a time from wherever they sit (ds_write2_b32, as store_item): as a float4 store the compiler
    // first assembled the quad in consecutive registers.
    const uint32_t slot_addr = lds_addr(&w.rec[R * lane_id]);
    auto put_result = [&](int k, float4 v) {
        if (k == 0) {
            lds_write2<0>(slot_addr, v.x, v.y);
            lds_write2<2>(slot_addr, v.z, v.w);
        } else {
            lds_write2<4>(slot_addr, v.x, v.y);
            lds_write2<6>(slot_addr, v.z, v.w);
        }
    };
    // The lanes whose first pixel is done (divergent): read the second record, then hand the first result to the slot
    // it came from (the sums are still in acc / accx), then start the second pixel's sums.
    auto next_pixel = [&]() {
        cur = load_item_any<EXACT>(&w.rec[R * lane_id]);
        m = ((uint64_t)cur.live1 << 32) | cur.live0;
        put_result(0, result());
        acc = splat3(0.0f, 0.0f, 0.0f);
        accx = mk3(0.0f, 0.0f, 0.0f);
    };
    // First pixels without a live light: hand them back and start the second ones at once (which may have none
    // either: then they are handed back too, and those lanes run sentinels only). `zero`: the lanes whose current
    // mask is empty, formed by ONE compare per iteration (at its end: the next iteration's live lanes are the rest).
    uint64_t zero = lanes(m == 0);
    if (zero != 0) {  // uniform
        if (on(zero)) next_pixel();
        second = zero;
        const uint64_t first_done = zero;
        zero = lanes(m == 0);
        const uint64_t empty = first_done & zero;
        if (empty != 0 && on(empty)) put_result(1, result());
    }
#if PBR_BAL_PROFILE
    int iters = 0;
#endif
    {
        // Lanes outside EXEC are never live: a ballot reports 0 for them, so ~zero alone would keep them live forever
        // under a partial EXEC (today's callers run this with the full wave; the mask costs one scalar op).
        const uint64_t exec = __builtin_amdgcn_read_exec();
        uint64_t live = ~zero & exec;
        while (live != 0) {
#if PBR_BAL_PROFILE
            ++iters;
#endif
            // Two live lights per lane (ctz saturating to the sentinel index: v_ffbl of 0 is -1), or the sentinel.
            const int j0 = m != 0 ? __builtin_ctzll(m) : kBalMaxLights;
            m &= m - 1;  // no-op when m == 0
            const int j1 = m != 0 ? __builtin_ctzll(m) : kBalMaxLights;
            m &= m - 1;
            m2 oki = m2{~0ull, ~0ull};  // this item pair's window tests, as lane masks
            f3x2 lp, ls;
            read_pair_lights(lds_lights, j0, j1, lp, ls);
            if constexpr (EXACT) {
                const f3x2 c = exact_point_items2(cur, lp, ls, oki, live);
                accx = mk3((accx.x + c.x.x) + c.x.y, (accx.y + c.y.x) + c.y.y, (accx.z + c.z.x) + c.z.y);
            } else {
                faithful_point_items2(cur, lp, ls, oki, acc, live);
            }
            fail |= ~(oki.x & oki.y) & live;
            // The lanes whose pixel just ran out of live lights.
            zero = lanes(m == 0);
            const uint64_t done = zero & live;
            if (done != 0) {  // uniform
                if (on(done)) {
                    if (on(second)) put_result(1, result());
                    if (!on(second)) next_pixel();
                }
                fail &= ~done;
                const uint64_t first_done = done & ~second;
                second |= first_done;
                if (first_done != 0) {  // those lanes hold their second pixel's mask now
                    zero = lanes(m == 0);
                    // A second pixel with no live light: hand it back now (rare).
                    const uint64_t empty = first_done & zero;
                    if (empty != 0 && on(empty)) put_result(1, result());
                }
            }
            live = ~zero & exec;
        }
    }
    BAL_PROF_T(t3);
    PBR_PHASE("handback");
    // ---- hand the results back: the owner reads its two pixels' from their evaluating lanes' slots (rank r < 64:
    // lane r, first pixel; r >= 64: lane 127 - r, second pixel)
    wave_lds_sync();
    const int2 rk = w.rank[lane_id];
    auto slot = [&](int r) {
        r = PBR_BOUNDS(r, 128, kBoundsLds);
        return r < 64 ? R * r : R * (127 - r) + 1;
    };
    const float4 ra = w.rec[slot(rk.x)], rb = w.rec[slot(rk.y)];
    wave_lds_sync();
    if constexpr (EXACT)
        sum = f3x2{v2{ra.x, rb.x}, v2{ra.y, rb.y}, v2{ra.z, rb.z}};
    else
        sum = f3x2{sum.x + v2{ra.x, rb.x}, sum.y + v2{ra.y, rb.y}, sum.z + v2{ra.z, rb.z}};
    redo |= mask2(live_a && ra.w == 0.0f, live_b && rb.w == 0.0f);
#if PBR_BAL_PROFILE
    BAL_PROF_T(t4);
    BAL_PROF_ADD(1, t2 - t1);
    BAL_PROF_ADD(2, t3 - t2);
    BAL_PROF_ADD(3, t4 - t3);
    BAL_PROF_ADD(4, 1);
    BAL_PROF_ADD(5, iters);
#endif
}

}  // namespace pbr
