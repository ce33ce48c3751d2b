// pbr_render.cpp -- native (C++, no Python) driver of the shading hot path through include/pbr/pbr_shade.hpp:
// the BASELINE scenes' G-buffer filled on the host (pbr_gbuffer_fill, the rasteriser front-end's stand-in),
// uploaded once to HBM, the pass constants of the scene, then the gfx950 shading pass -- once, as row bands
// (the multi-GPU partition's pointer offsets), or timed with HIP events like bench.py.
//
//   hipcc -std=c++17 -O2 -I include examples/pbr_render.cpp -L physically_based_renderer_amd/_lib -lpbrshade \
//         -lz -Wl,-rpath,$PWD/physically_based_renderer_amd/_lib -o build/pbr_render
//   build/pbr_render --config 3 --steps 50            # timed: one JSON line (--mode faithful: PBR_FLAG_FAITHFUL)
//   build/pbr_render --config 2 --dump frame.bin      # one frame -> file (tests compare it with the oracle)
//   build/pbr_render --check-assets                   # decode the assets only (no GPU)
//
// Scenes (same table as physically_based_renderer_amd/scenes.py CONFIGS): 1 rustediron sphere, 1 point light;
// 2 1920x1080, 8 point lights; 3 3840x2160, 64 point lights + diffuse IBL; 4 3840x2160, 256 point lights,
// tiled culling, material tiles + F0 plane; 5 8192x8192, 64 point lights + IBL.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "asset_io.hpp"
#include "pbr/pbr_shade.hpp"

namespace {

struct SceneConfig {
    int id;
    const char* name;
    int kind, width, height, n_lights;
    pbr::AmbientMode ambient;
    uint32_t flags;
    uint64_t seed;
};

const SceneConfig kConfigs[] = {
    {1, "cfg1_256x256_sphere_rustediron_1pt", PBR_SCENE_SPHERE_RUSTEDIRON, 256, 256, 1, pbr::AmbientMode::Constant, 0,
     0x5EED0001ull},
    {2, "cfg2_1920x1080_rustediron_8pt", PBR_SCENE_RANDOM_COVERED, 1920, 1080, 8, pbr::AmbientMode::Constant, 0,
     0x5EED0002ull},
    {3, "cfg3_3840x2160_64pt_ibl_chelsea", PBR_SCENE_RANDOM_COVERED, 3840, 2160, 64, pbr::AmbientMode::IblDiffuse, 0,
     0x5EED0003ull},
    {4, "cfg4_3840x2160_256pt_tiled_materials", PBR_SCENE_PLANE_MATERIALS, 3840, 2160, 256, pbr::AmbientMode::Constant,
     PBR_FLAG_F0_PLANE | PBR_FLAG_TILED_CULLING, 0x5EED0004ull},
    {5, "cfg5_8192x8192_64pt_ibl_rowbands", PBR_SCENE_RANDOM_COVERED, 8192, 8192, 64, pbr::AmbientMode::IblDiffuse, 0,
     0x5EED0005ull},
};

uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

// The committed texture tiles and environment (physically_based_renderer_amd/assets, tools/make_assets.py).
struct Assets {
    std::map<std::string, pbr_assets::U8Array> rust, mats;
    pbr_assets::Rgba16Image env;
    pbr_scene_assets c{};

    explicit Assets(const std::string& dir) {
        rust = pbr_assets::load_npz_u8(dir + "/rustediron_256.npz", {"metallic", "roughness"});
        mats = pbr_assets::load_npz_u8(dir + "/materials_1k_64.npz",
                                       {"albedo", "specular", "roughness", "metallic", "has_metallic", "normal"});
        env = pbr_assets::decode_png_rgba16(dir + "/Chelsea_Stairs_Env.png");
        c.rust_metallic = rust["metallic"].data.data();
        c.rust_roughness = rust["roughness"].data.data();
        c.rust_size = static_cast<int32_t>(rust["metallic"].shape.at(0));
        c.mat_albedo = mats["albedo"].data.data();
        c.mat_specular = mats["specular"].data.data();
        c.mat_roughness = mats["roughness"].data.data();
        c.mat_metallic = mats["metallic"].data.data();
        c.mat_has_metallic = mats["has_metallic"].data.data();
        c.mat_normal = mats["normal"].data.data();
        c.num_materials = static_cast<int32_t>(mats["albedo"].shape.at(0));
        c.mat_size = static_cast<int32_t>(mats["albedo"].shape.at(1));
    }
};

struct Args {
    int config = 3, width = 0, height = 0, steps = 0, warmup = 3, bands = 1, threads = 0;
    double ramp_ms = 200.0;
    std::string output = "rgba32f", mode = "exact", dump, assets = "physically_based_renderer_amd/assets";
    bool check_assets = false;
};

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + k);
            return argv[++i];
        };
        if (k == "--config") a.config = std::stoi(val());
        else if (k == "--width") a.width = std::stoi(val());
        else if (k == "--height") a.height = std::stoi(val());
        else if (k == "--steps") a.steps = std::stoi(val());
        else if (k == "--warmup") a.warmup = std::stoi(val());
        else if (k == "--bands") a.bands = std::stoi(val());
        else if (k == "--threads") a.threads = std::stoi(val());
        else if (k == "--ramp-ms") a.ramp_ms = std::stod(val());
        else if (k == "--output") a.output = val();
        else if (k == "--mode") a.mode = val();
        else if (k == "--dump") a.dump = val();
        else if (k == "--assets") a.assets = val();
        else if (k == "--check-assets") a.check_assets = true;
        else throw std::runtime_error("unknown option " + k);
    }
    if (a.output != "rgba32f" && a.output != "rgba8") throw std::runtime_error("--output rgba32f|rgba8");
    if (a.mode != "exact" && a.mode != "faithful") throw std::runtime_error("--mode exact|faithful");
    if (a.bands < 1) throw std::runtime_error("--bands >= 1");
    return a;
}

int run(const Args& args) {
    Assets assets(args.assets);
    if (args.check_assets) {  // decode only: checksums the CPU test compares with numpy's decode
        for (const auto& set : {std::make_pair("rustediron_256", &assets.rust), std::make_pair("materials_1k_64", &assets.mats)})
            for (const auto& kv : *set.second)
                std::printf("%s/%s %016llx\n", set.first, kv.first.c_str(),
                            (unsigned long long)fnv1a(kv.second.data.data(), kv.second.data.size()));
        std::printf("env %dx%d %016llx\n", assets.env.width, assets.env.height,
                    (unsigned long long)fnv1a(reinterpret_cast<const uint8_t*>(assets.env.texels.data()),
                                              assets.env.texels.size() * sizeof(uint16_t)));
        return 0;
    }
    const SceneConfig* cfg = nullptr;
    for (const auto& c : kConfigs)
        if (c.id == args.config) cfg = &c;
    if (!cfg) throw std::runtime_error("--config 1..5");
    const int W = args.width ? args.width : cfg->width, H = args.height ? args.height : cfg->height;
    const int threads = args.threads ? args.threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));

    // Host fill: pixel values depend on (global x, y, seed) only (pbr_gbuffer_fill).
    pbr_scene_desc scene;
    std::memset(&scene, 0, sizeof scene);
    scene.kind = cfg->kind;
    scene.width = W;
    scene.height = H;
    scene.seed = cfg->seed;
    scene.assets = &assets.c;
    const size_t plane = static_cast<size_t>(W) * H;
    float* host = nullptr;
    PBR_THROW_IF_HIP(hipHostMalloc(reinterpret_cast<void**>(&host), sizeof(float) * pbr::DeviceGBuffer::kPlanes * plane));
    float* planes[pbr::DeviceGBuffer::kPlanes];
    for (int i = 0; i < pbr::DeviceGBuffer::kPlanes; ++i) planes[i] = host + i * plane;
    const auto t0 = std::chrono::steady_clock::now();
    PBR_THROW_IF_FAILED(pbr_gbuffer_fill(&scene, 0, H, planes, W, threads));
    const double fill_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    // The scene's pass (UpdateMainPassCB's role): lights + constants, then the config's ambient and flags.
    std::vector<pbr_light> lights(std::max(cfg->n_lights, 1));
    pbr_pass_desc pass;
    PBR_THROW_IF_FAILED(pbr_scene_pass(&scene, cfg->n_lights, lights.data(), &pass));
    pass.ambient_mode = static_cast<int32_t>(cfg->ambient);
    pass.flags |= cfg->flags;
    if (args.mode == "faithful") pass.flags |= PBR_FLAG_FAITHFUL;  // tolerance mode (pbr_shade.h)

    hipStream_t stream;
    PBR_THROW_IF_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    pbr::ShadingContext ctx(0);
    pbr::DeviceGBuffer gb(W, H);
    gb.Upload(host, stream);
    ctx.SetPass(pass, stream);
    if (cfg->ambient == pbr::AmbientMode::IblDiffuse) ctx.SetEnvMap(assets.env.texels.data(), assets.env.width, assets.env.height, stream);

    const bool rgba8 = args.output == "rgba8";
    const size_t px_bytes = rgba8 ? 4 : 16;
    void* out = nullptr;
    PBR_THROW_IF_HIP(hipMalloc(&out, px_bytes * plane));
    const pbr_output_format fmt = rgba8 ? PBR_OUTPUT_RGBA8_UNORM : PBR_OUTPUT_RGBA32F;

    // One pass = the frame as `bands` row bands (8-row aligned like dist.band_rows), each shaded through
    // pointers offset to its first row, as one GPU of a row-partitioned frame does.
    auto shade = [&]() {
        const int tiles = (H + 7) / 8, per = tiles / args.bands, extra = tiles % args.bands;
        int r0 = 0;
        for (int b = 0; b < args.bands; ++b) {
            const int r1 = std::min(H, r0 + 8 * (per + (b >= args.bands - extra ? 1 : 0)));
            if (r1 > r0) {
                const pbr_gbuffer_soa band = gb.Band(r0, r1);
                void* dst = static_cast<uint8_t*>(out) + px_bytes * static_cast<size_t>(r0) * W;
                ctx.ShadeFrame(band, dst, W, fmt, nullptr, 0, stream);
            }
            r0 = r1;
        }
    };

    if (args.steps <= 0) {
        shade();
        PBR_THROW_IF_HIP(hipStreamSynchronize(stream));
        std::vector<uint8_t> frame(px_bytes * plane);
        PBR_THROW_IF_HIP(hipMemcpy(frame.data(), out, frame.size(), hipMemcpyDeviceToHost));
        const pbr_pass_stats st = ctx.LastPassStats(stream);
        if (!args.dump.empty()) {  // int32 W, H, bytes per pixel, 0; then the frame
            FILE* f = std::fopen(args.dump.c_str(), "wb");
            if (!f) throw std::runtime_error("cannot write " + args.dump);
            const int32_t hdr[4] = {W, H, static_cast<int32_t>(px_bytes), 0};
            std::fwrite(hdr, sizeof hdr, 1, f);
            std::fwrite(frame.data(), 1, frame.size(), f);
            std::fclose(f);
        }
        std::printf("{\"tool\": \"pbr_render\", \"workload\": \"%s\", \"width\": %d, \"height\": %d, \"bands\": %d, "
                    "\"output\": \"%s\", \"mode\": \"%s\", \"fnv1a\": \"%016llx\", \"exact_pixels\": %lld, \"fill_s\": %.3f}\n",
                    cfg->name, W, H, args.bands, args.output.c_str(), args.mode.c_str(),
                    (unsigned long long)fnv1a(frame.data(), frame.size()),
                    (long long)st.exact_pixels, fill_s);
    } else {
        // Clock ramp (untimed back-to-back passes, as bench.py), warm-up, then `steps` passes each bracketed
        // by HIP events on the launch stream; the wall clock spans all of them between synchronisations.
        const auto tr = std::chrono::steady_clock::now();
        int ramp = 0;
        while (args.ramp_ms > 0) {
            shade();
            if (++ramp % 8 == 0) {
                PBR_THROW_IF_HIP(hipStreamSynchronize(stream));
                if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count() >= args.ramp_ms) break;
            }
        }
        for (int i = 0; i < args.warmup; ++i) shade();
        PBR_THROW_IF_HIP(hipStreamSynchronize(stream));
        std::vector<hipEvent_t> ev(2 * args.steps);
        for (auto& e : ev) PBR_THROW_IF_HIP(hipEventCreate(&e));
        const auto ts = std::chrono::steady_clock::now();
        for (int i = 0; i < args.steps; ++i) {
            PBR_THROW_IF_HIP(hipEventRecord(ev[2 * i], stream));
            shade();
            PBR_THROW_IF_HIP(hipEventRecord(ev[2 * i + 1], stream));
        }
        PBR_THROW_IF_HIP(hipStreamSynchronize(stream));
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
        std::vector<float> ms(args.steps);
        for (int i = 0; i < args.steps; ++i) PBR_THROW_IF_HIP(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
        for (auto& e : ev) (void)hipEventDestroy(e);
        double mean = 0;
        for (float m : ms) mean += m;
        mean /= args.steps;
        std::vector<float> sorted = ms;
        std::sort(sorted.begin(), sorted.end());
        std::printf("{\"tool\": \"pbr_render\", \"workload\": \"%s\", \"width\": %d, \"height\": %d, \"bands\": %d, "
                    "\"output\": \"%s\", \"mode\": \"%s\", \"steps\": %d, \"value\": %.2f, \"unit\": \"Mpix/s\", \"ms_per_step\": %.4f, "
                    "\"event_mean_ms\": %.4f, \"event_median_ms\": %.4f, \"clock_ramp_launches\": %d}\n",
                    cfg->name, W, H, args.bands, args.output.c_str(), args.mode.c_str(), args.steps, static_cast<double>(plane) * args.steps / wall / 1e6,
                    wall / args.steps * 1e3, mean, sorted[args.steps / 2], ramp);
    }
    PBR_THROW_IF_HIP(hipFree(out));
    PBR_THROW_IF_HIP(hipHostFree(host));
    PBR_THROW_IF_HIP(hipStreamDestroy(stream));
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        return run(parse(argc, argv));
    } catch (const pbr::ShadeException& e) {
        std::fprintf(stderr, "pbr_render: %s\n", e.ToString().c_str());
        return 1;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "pbr_render: %s\n", e.what());
        return 2;
    }
}
