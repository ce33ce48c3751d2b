// oracle/hlsl_prelude.hpp -- TEST INFRASTRUCTURE ONLY.
//
// The HLSL *language* built-ins (vector/matrix types, swizzles, operators, intrinsics) as C++, so that
// the reference's own shader text compiles with g++: LightingUtil.hlsl unmodified, and Core.hlsl /
// Default.hlsl / Skybox.hlsl after oracle/strip_hlsl.py's syntax-only rewrite. No reference header,
// library or generated file is replaced; resource types (Texture2D, SamplerState) are bound by
// oracle/ref_harness.cpp.
// Semantics follow HLSL SM5 / D3D10+ fp32 rules:
//   * literals are fp32 (build with -fsingle-precision-constant: HLSL has no implicit double);
//   * per-component IEEE ops, no contraction (-ffp-contract=off);
//   * dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z; normalize(v) = v / sqrt(dot(v,v));
//   * max/min are IEEE maxNum/minNum (a NaN operand yields the other one); saturate(NaN) = 0;
//   * lerp(x, y, s) = x + s*(y - x); pow/atan2/asin come from libm;
//   * a wider vector converts to a narrower one by truncation (float4 -> float3 keeps .xyz, float3 ->
//     float2 keeps .xy), as HLSL's implicit conversions do (Default.hlsl:150, Skybox.hlsl:43).
#pragma once
#include <cmath>

namespace hlsl {

struct float2 {
    float x, y;
    float2() : x(0.0f), y(0.0f) {}
    float2(float s) : x(s), y(s) {}
    float2(float a, float b) : x(a), y(b) {}
};
inline float2 operator+(float2 a, float2 b) { return float2(a.x + b.x, a.y + b.y); }
inline float2 operator*(float2 a, float2 b) { return float2(a.x * b.x, a.y * b.y); }

struct float3 {
    float x, y, z;
    float3() : x(0.0f), y(0.0f), z(0.0f) {}
    float3(float s) : x(s), y(s), z(s) {}
    float3(float a, float b, float c) : x(a), y(b), z(c) {}
    float3& operator+=(const float3& o) { x += o.x; y += o.y; z += o.z; return *this; }
    float3& operator-=(const float3& o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    float3& operator*=(const float3& o) { x *= o.x; y *= o.y; z *= o.z; return *this; }
    float3& operator/=(const float3& o) { x /= o.x; y /= o.y; z /= o.z; return *this; }
    float3 rgb() const { return *this; }
    operator float2() const { return float2(x, y); }  // implicit truncation
};
inline float3 operator+(float3 a, float3 b) { return float3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline float3 operator-(float3 a, float3 b) { return float3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline float3 operator*(float3 a, float3 b) { return float3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline float3 operator/(float3 a, float3 b) { return float3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline float3 operator-(float3 a) { return float3(-a.x, -a.y, -a.z); }
inline float3 operator+(float3 a, float s) { return a + float3(s); }
inline float3 operator+(float s, float3 a) { return float3(s) + a; }
inline float3 operator-(float3 a, float s) { return a - float3(s); }
inline float3 operator-(float s, float3 a) { return float3(s) - a; }
inline float3 operator*(float3 a, float s) { return a * float3(s); }
inline float3 operator*(float s, float3 a) { return float3(s) * a; }
inline float3 operator/(float3 a, float s) { return a / float3(s); }
inline float3 operator/(float s, float3 a) { return float3(s) / a; }

// Swizzle as an lvalue (Skybox.hlsl:29 `posW.xyz += g_CameraPosW`).
struct swizzle3 {
    float &a, &b, &c;
    operator float3() const { return float3(a, b, c); }
    swizzle3& operator+=(float3 v) { a += v.x; b += v.y; c += v.z; return *this; }
};

struct float4 {
    float x, y, z, w;
    float4() : x(0.0f), y(0.0f), z(0.0f), w(0.0f) {}
    float4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    float4(float3 v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
    float4(float2 v, float c, float d) : x(v.x), y(v.y), z(c), w(d) {}
    operator float3() const { return float3(x, y, z); }  // implicit truncation
    float3 rgb() const { return float3(x, y, z); }
    float r() const { return x; }
    float2 xy() const { return float2(x, y); }
    swizzle3 xyz() { return swizzle3{x, y, z}; }
    float4 xyww() const { return float4(x, y, w, w); }
};
// float3x3(r0, r1, r2) builds rows; mul(rowvector, M) = sum_i v[i] * M[i].
struct float3x3 {
    float3 r0, r1, r2;
    float3x3(float3 a, float3 b, float3 c) : r0(a), r1(b), r2(c) {}
};
inline float3 mul(float3 v, float3x3 m) { return v.x * m.r0 + v.y * m.r1 + v.z * m.r2; }

// float4x4 (row-major rows, as the app's XMStoreFloat4x4(XMMatrixTranspose(..)) uploads them) and
// mul(float4 row vector, float4x4); `(float3x3)m` keeps the upper-left 3x3 (Default.hlsl:31).
struct float4x4 {
    float4 r0, r1, r2, r3;
    explicit operator float3x3() const { return float3x3(r0, r1, r2); }
};
inline float4 operator*(float s, float4 a) { return float4(s * a.x, s * a.y, s * a.z, s * a.w); }
inline float4 operator+(float4 a, float4 b) { return float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
inline float4 mul(float4 v, float4x4 m) { return v.x * m.r0 + v.y * m.r1 + v.z * m.r2 + v.w * m.r3; }

inline float dot(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float length(float3 a) { return std::sqrt(dot(a, a)); }
inline float3 normalize(float3 a) { return a / std::sqrt(dot(a, a)); }
inline float max(float a, float b) { return std::fmax(a, b); }
inline float min(float a, float b) { return std::fmin(a, b); }
inline float saturate(float a) { return std::fmin(std::fmax(a, 0.0f), 1.0f); }
inline float pow(float a, float b) { return std::pow(a, b); }
inline float3 pow(float3 a, float b) { return float3(std::pow(a.x, b), std::pow(a.y, b), std::pow(a.z, b)); }
inline float atan2(float y, float x) { return std::atan2(y, x); }
inline float asin(float a) { return std::asin(a); }
inline float lerp(float x, float y, float s) { return x + s * (y - x); }
inline float3 lerp(float3 x, float3 y, float s) { return x + s * (y - x); }
// clip(x): discard the fragment when x < 0 (Default.hlsl:113, ALPHA_TEST permutations only): the harness
// clears the flag before each pixel and leaves a discarded pixel's output untouched (ref_harness.cpp).
inline thread_local bool g_clip_discarded = false;
inline void clip(float x) { if (x < 0.0f) g_clip_discarded = true; }

}  // namespace hlsl
