// oracle/hlsl_prelude.hpp -- TEST INFRASTRUCTURE ONLY.
//
// The HLSL *language* built-ins (vector types, operators, intrinsics) as C++, so that the reference's
// own shader text, /root/reference/Source/Shaders/LightingUtil.hlsl, compiles unmodified with g++.
// No reference header, library or generated file is replaced: LightingUtil.hlsl includes nothing.
// Semantics follow HLSL SM5 / D3D10+ fp32 rules:
//   * literals are fp32 (build with -fsingle-precision-constant: HLSL has no implicit double);
//   * per-component IEEE ops, no contraction (-ffp-contract=off);
//   * dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z; normalize(v) = v / sqrt(dot(v,v));
//   * max/min are IEEE maxNum/minNum (a NaN operand yields the other one); saturate(NaN) = 0;
//   * lerp(x, y, s) = x + s*(y - x); pow/atan2/asin come from libm.
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

struct float4 {
    float x, y, z, w;
    float3 rgb() const { return float3(x, y, z); }
};

// float3x3(r0, r1, r2) builds rows; mul(rowvector, M) = sum_i v[i] * M[i].
struct float3x3 {
    float3 r0, r1, r2;
    float3x3(float3 a, float3 b, float3 c) : r0(a), r1(b), r2(c) {}
};
inline float3 mul(float3 v, float3x3 m) { return v.x * m.r0 + v.y * m.r1 + v.z * m.r2; }

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

}  // namespace hlsl
