// pbr_shade.hpp -- C++17 host interface over the C ABI of libpbrshade.so (include/pbr/pbr_shade.h).
//
// The reference renderer is C++ (Source/App), so this is the host side a maintainer of it would use:
// the same types and roles as the reference's own shading interface, with its error behaviour.
//
//   reference                                              here
//   -----------------------------------------------------  ------------------------------------------
//   struct Light (d3dUtil.h:144-152)                        pbr::Light (same fields, defaults, 48 bytes)
//   PassConstants::EyePosW / AmbientLight / Lights          pbr::PassConstants (FrameResource.h:19-44)
//     + NUM_DIR/POINT/SPOT_LIGHTS defines (Core.hlsl:1-11)    (counts are runtime values here)
//   MaterialProperties::FresnelR0 / Opacity (Material.h)    pbr::MaterialProperties
//   DxException + ThrowIfFailed (d3dUtil.h:130-163)         pbr::ShadeException + PBR_THROW_IF_FAILED
//   device/PSO creation, UpdateMainPassCB, DrawIndexed      pbr::ShadingContext (RAII over pbr_context)
//   the G-buffer render targets the lit pass reads          pbr::DeviceGBuffer (15 SoA planes in HBM)
//
// Nothing here computes: every shading call is the gfx950 kernel behind the C ABI. Header-only; link
// libpbrshade.so and libamdhip64.so.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "pbr/pbr_shade.h"

namespace pbr {

struct float3 {
    float x = 0.0f, y = 0.0f, z = 0.0f;
};
struct float4 {
    float x = 0.0f, y = 0.0f, z = 0.0f, w = 0.0f;
};

// struct Light (d3dUtil.h:144-152; HLSL LightingUtil.hlsl:9-17): the reference's defaults, byte layout
// identical to pbr_light, so an array of either passes through unchanged.
struct Light {
    float3 Strength = {0.5f, 0.5f, 0.5f};
    float SpotPower = 64.0f;                 // spot light only
    float3 Direction = {0.0f, -1.0f, 0.0f};  // directional / spot light only
    float __PAD000 = 0.0f;
    float3 Position = {0.0f, 0.0f, 0.0f};    // point / spot light only
    float __PAD001 = 0.0f;
};
static_assert(sizeof(Light) == sizeof(pbr_light) && sizeof(Light) == 48, "Light must stay the 48-byte cbuffer element");
static_assert(offsetof(Light, Direction) == offsetof(pbr_light, direction) &&
                  offsetof(Light, Position) == offsetof(pbr_light, position) &&
                  offsetof(Light, SpotPower) == offsetof(pbr_light, spot_power),
              "Light layout drifted from pbr_light");

enum class AmbientMode : int32_t {
    Constant = PBR_AMBIENT_CONSTANT,     // g_AmbientLight * albedo (Default.hlsl:150)
    IblDiffuse = PBR_AMBIENT_IBL_DIFFUSE // the diffuse-IBL block (Default.hlsl:140-149)
};

// The shading subset of PassConstants (FrameResource.h:19-44). Lights are ordered directional, point,
// spot, as ComputeLighting walks them (LightingUtil.hlsl:176-199); unlike the reference's fixed
// Lights[MaxLights = 16] the list holds up to PBR_MAX_LIGHTS.
struct PassConstants {
    float3 EyePosW = {0.0f, 0.0f, 0.0f};
    float4 AmbientLight = {0.0f, 0.0f, 0.0f, 1.0f};
    std::vector<Light> Lights;
    int32_t NumDirLights = 0;
    int32_t NumPointLights = 0;
    int32_t NumSpotLights = 0;
    AmbientMode Ambient = AmbientMode::Constant;
    uint32_t Flags = 0;  // pbr_pass_flags
};

// The two MaterialProperties fields PS reads outside the G-buffer (Material.h:10-29, Default.hlsl:94-95, 160).
struct MaterialProperties {
    float3 FresnelR0 = {0.04f, 0.04f, 0.04f};
    float Opacity = 1.0f;
};

// DxException (d3dUtil.h:130-143): the failing call, file and line; ToString() like the reference's.
class ShadeException : public std::runtime_error {
  public:
    ShadeException(int code, const std::string& function, const std::string& file, int line, const std::string& detail)
        : std::runtime_error(Format(code, function, file, line, detail)), ErrorCode(code), FunctionName(function),
          Filename(file), LineNumber(line) {}
    std::string ToString() const { return what(); }

    int ErrorCode = PBR_OK;
    std::string FunctionName;
    std::string Filename;
    int LineNumber = -1;

  private:
    static std::string Format(int code, const std::string& fn, const std::string& file, int line, const std::string& d) {
        std::string s = fn + " failed in " + file + "; line " + std::to_string(line) + "; error: " + pbr_strerror(code);
        if (!d.empty()) s += " (" + d + ")";
        return s;
    }
};

namespace detail {
inline void throw_if_failed(int64_t status, const char* expr, const char* file, int line,
                            const pbr_context* ctx = nullptr) {
    if (status < 0) throw ShadeException(static_cast<int>(status), expr, file, line, ctx ? pbr_last_error(ctx) : "");
}
inline void throw_if_hip(hipError_t e, const char* expr, const char* file, int line) {
    if (e != hipSuccess) throw ShadeException(PBR_ERR_HIP, expr, file, line, hipGetErrorString(e));
}
}  // namespace detail

// ThrowIfFailed (d3dUtil.h:156-163) for pbr_* status codes and HIP calls.
#define PBR_THROW_IF_FAILED(x) ::pbr::detail::throw_if_failed((x), #x, __FILE__, __LINE__)
#define PBR_THROW_IF_HIP(x) ::pbr::detail::throw_if_hip((x), #x, __FILE__, __LINE__)

// The lit pass's inputs in HBM: 15 fp32 planes (pos xyz, normal xyz, albedo rgb, metallic, roughness,
// AO, F0 rgb), `row_stride` floats per row, one allocation. Owned here; the library only reads it.
class DeviceGBuffer {
  public:
    static constexpr int kPlanes = 15;

    DeviceGBuffer() = default;
    DeviceGBuffer(int32_t width, int32_t height) : width_(width), height_(height), row_stride_(width) {
        if (width <= 0 || height < 0) throw ShadeException(PBR_ERR_INVALID_ARGUMENT, "DeviceGBuffer", __FILE__, __LINE__, "size");
        PBR_THROW_IF_HIP(hipMalloc(reinterpret_cast<void**>(&planes_), bytes()));
    }
    DeviceGBuffer(const DeviceGBuffer&) = delete;
    DeviceGBuffer& operator=(const DeviceGBuffer&) = delete;
    DeviceGBuffer(DeviceGBuffer&& o) noexcept { *this = std::move(o); }
    DeviceGBuffer& operator=(DeviceGBuffer&& o) noexcept {
        std::swap(planes_, o.planes_);
        std::swap(width_, o.width_);
        std::swap(height_, o.height_);
        std::swap(row_stride_, o.row_stride_);
        return *this;
    }
    ~DeviceGBuffer() {
        if (planes_) (void)hipFree(planes_);
    }

    int32_t width() const { return width_; }
    int32_t height() const { return height_; }
    int64_t row_stride() const { return row_stride_; }
    size_t bytes() const { return sizeof(float) * kPlanes * static_cast<size_t>(row_stride_) * height_; }
    float* plane(int i) { return planes_ + static_cast<size_t>(i) * row_stride_ * height_; }
    const float* plane(int i) const { return planes_ + static_cast<size_t>(i) * row_stride_ * height_; }

    // Upload host planes laid out like this buffer (plane-major, width floats per row).
    void Upload(const float* host, hipStream_t stream = nullptr) {
        PBR_THROW_IF_HIP(hipMemcpyAsync(planes_, host, bytes(), hipMemcpyHostToDevice, stream));
    }

    // Rows [row_begin, row_end) as a pbr_gbuffer_soa: pointers offset to the band, so shading it is the
    // multi-GPU row tile (the result equals the same rows of a whole-frame pass).
    pbr_gbuffer_soa Band(int32_t row_begin, int32_t row_end) const {
        if (row_begin < 0 || row_end < row_begin || row_end > height_)
            throw ShadeException(PBR_ERR_INVALID_ARGUMENT, "DeviceGBuffer::Band", __FILE__, __LINE__, "rows");
        pbr_gbuffer_soa g;
        std::memset(&g, 0, sizeof g);
        const size_t off = static_cast<size_t>(row_begin) * row_stride_;
        for (int k = 0; k < 3; ++k) {
            g.pos_w[k] = plane(0 + k) + off;
            g.normal_w[k] = plane(3 + k) + off;
            g.albedo[k] = plane(6 + k) + off;
            g.f0[k] = plane(12 + k) + off;
        }
        g.metallic = plane(9) + off;
        g.roughness = plane(10) + off;
        g.ao = plane(11) + off;
        g.opacity = nullptr;  // PBR_FLAG_ALPHA_TEST: set it to an opacity plane with this row stride
        g.width = width_;
        g.height = row_end - row_begin;
        g.row_stride = row_stride_;
        return g;
    }
    pbr_gbuffer_soa View() const { return Band(0, height_); }

  private:
    float* planes_ = nullptr;
    int32_t width_ = 0, height_ = 0;
    int64_t row_stride_ = 0;
};

// One device's shading pipeline: replaces device + PSO creation (d3dApp.cpp:437-501, PBRApp.cpp:607-650,
// 776-881), UpdateMainPassCB (PBRApp.cpp:455-502), the sky/env SRVs (PBRApp.cpp:1200-1210) and the lit
// pass's DrawIndexedInstanced (PBRApp.cpp:1133). Calls are asynchronous on the stream given.
class ShadingContext {
  public:
    explicit ShadingContext(int device = 0) {
        PBR_THROW_IF_FAILED(pbr_context_create(device, &ctx_));
    }
    ShadingContext(const ShadingContext&) = delete;
    ShadingContext& operator=(const ShadingContext&) = delete;
    ~ShadingContext() {
        if (ctx_) (void)pbr_context_destroy(ctx_);
    }
    pbr_context* get() const { return ctx_; }

    // UpdateMainPassCB + CopyData: the light list and constants, stream-ordered (`pass` reusable on return).
    void SetPass(const PassConstants& pass, const MaterialProperties& mat = {}, hipStream_t stream = nullptr) {
        const size_t n = static_cast<size_t>(pass.NumDirLights) + pass.NumPointLights + pass.NumSpotLights;
        if (pass.Lights.size() < n)
            throw ShadeException(PBR_ERR_INVALID_ARGUMENT, "ShadingContext::SetPass", __FILE__, __LINE__,
                                 std::to_string(n) + " lights declared, " + std::to_string(pass.Lights.size()) + " given");
        pbr_pass_desc d;
        std::memset(&d, 0, sizeof d);
        const float eye[3] = {pass.EyePosW.x, pass.EyePosW.y, pass.EyePosW.z};
        const float amb[3] = {pass.AmbientLight.x, pass.AmbientLight.y, pass.AmbientLight.z};  // .rgb (Default.hlsl:150)
        const float f0[3] = {mat.FresnelR0.x, mat.FresnelR0.y, mat.FresnelR0.z};
        std::memcpy(d.eye_pos_w, eye, sizeof eye);
        std::memcpy(d.ambient_light, amb, sizeof amb);
        std::memcpy(d.fresnel_r0, f0, sizeof f0);
        d.opacity = mat.Opacity;
        d.num_dir_lights = pass.NumDirLights;
        d.num_point_lights = pass.NumPointLights;
        d.num_spot_lights = pass.NumSpotLights;
        d.ambient_mode = static_cast<int32_t>(pass.Ambient);
        d.flags = pass.Flags;
        d.lights = n ? reinterpret_cast<const pbr_light*>(pass.Lights.data()) : nullptr;
        Check(pbr_set_pass(ctx_, &d, stream), "pbr_set_pass");
    }
    void SetPass(const pbr_pass_desc& d, hipStream_t stream = nullptr) { Check(pbr_set_pass(ctx_, &d, stream), "pbr_set_pass"); }

    // g_SkyArray[1] (environment, R16G16B16A16_UNORM) and g_SkyArray[0] (sky box).
    void SetEnvMap(const uint16_t* texels, int32_t w, int32_t h, hipStream_t stream = nullptr) {
        Check(pbr_set_env_map(ctx_, texels, w, h, stream), "pbr_set_env_map");
    }
    void SetSkyMap(const uint16_t* texels, int32_t w, int32_t h, hipStream_t stream = nullptr) {
        Check(pbr_set_sky_map(ctx_, texels, w, h, stream), "pbr_set_sky_map");
    }

    // DrawIndexedInstanced(PS) over the G-buffer (or a band of it): fp32 RGBA into `out_rgba` (device).
    void Shade(const pbr_gbuffer_soa& gb, float* out_rgba, int64_t out_row_stride, hipStream_t stream = nullptr) {
        Check(pbr_shade_gbuffer(ctx_, &gb, out_rgba, out_row_stride, stream), "pbr_shade_gbuffer");
    }
    // The presented frame: lit geometry + sky dome where `coverage` is 0, fp32 or the R8G8B8A8_UNORM back buffer.
    void ShadeFrame(const pbr_gbuffer_soa& gb, void* out, int64_t out_row_stride, pbr_output_format format,
                    const uint8_t* coverage = nullptr, int64_t coverage_row_stride = 0, hipStream_t stream = nullptr) {
        pbr_frame_desc f;
        std::memset(&f, 0, sizeof f);
        f.out = out;
        f.out_row_stride = out_row_stride;
        f.format = format;
        f.coverage = coverage;
        f.coverage_row_stride = coverage_row_stride;
        Check(pbr_shade_frame(ctx_, &gb, &f, stream), "pbr_shade_frame");
    }

    pbr_pass_stats LastPassStats(hipStream_t stream = nullptr) {
        pbr_pass_stats s;
        Check(pbr_last_pass_stats(ctx_, &s, stream), "pbr_last_pass_stats");
        return s;
    }

  private:
    void Check(int status, const char* fn) {
        if (status < 0) throw ShadeException(status, fn, __FILE__, __LINE__, pbr_last_error(ctx_));
    }
    pbr_context* ctx_ = nullptr;
};

}  // namespace pbr
