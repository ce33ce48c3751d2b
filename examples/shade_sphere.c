/* examples/shade_sphere.c -- the C ABI (include/pbr/pbr_shade.h) used from plain C, the way the
 * reference renderer's own host code would call it:
 *
 *   1. the caller's "rasteriser front-end" fills a structure-of-arrays G-buffer: here a unit sphere
 *      at the origin ray-cast from the reference's initial camera (eye (0, 0, -5) looking down +z,
 *      fovY pi/4, PBRApp.cpp:652-659), with a red material whose roughness runs left to right and a
 *      coverage byte per pixel (0 = sky);
 *   2. the pass constants are the reference's (PBRApp.cpp:455-502): ambient 0.03 and its four
 *      directional lights (PBRApp.cpp:480-487);
 *   3. pbr_shade_frame writes the presented R8G8B8A8_UNORM frame (lit sphere + sky dome) on the GPU.
 *
 * Writes a binary PPM and prints an FNV-1a checksum of the RGBA8 frame. `--dump FILE` also writes the
 * host G-buffer, coverage, sky texels and frame (tests/test_c_example.py checks the frame against the
 * CPU oracle bit for bit).
 *
 *   gcc -std=c11 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include examples/shade_sphere.c \
 *       -L physically_based_renderer_amd/_lib -lpbrshade -L /opt/rocm/lib -lamdhip64 -lm \
 *       -Wl,-rpath,$PWD/physically_based_renderer_amd/_lib -o build/shade_sphere
 *   build/shade_sphere [--width 640 --height 360 --out sphere.ppm --dump frame.bin] [--host-only]
 */
#include <hip/hip_runtime_api.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pbr/pbr_shade.h"

#define NUM_PLANES 15
#define PI_D 3.14159265358979323846

static int check_pbr(int status, const char* what, const pbr_context* ctx) {
    if (status < 0) {
        fprintf(stderr, "%s: %s %s\n", what, pbr_strerror(status), ctx ? pbr_last_error(ctx) : "");
        exit(1);
    }
    return status;
}

static void check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

/* Ray-cast the unit sphere: per pixel position, normal, material, coverage (the G-buffer pass the
 * reference's rasteriser + VS would produce; Default.hlsl:22-45). Background pixels carry the view
 * ray in their normal planes (the sky dome direction, Skybox.hlsl:24). */
static void fill_gbuffer(int w, int h, float* planes, uint8_t* coverage) {
    const size_t n = (size_t)w * h;
    const double tan_half = tan(PI_D / 8.0), aspect = (double)w / h;
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            const size_t i = (size_t)y * w + x;
            double dx = (2.0 * (x + 0.5) / w - 1.0) * tan_half * aspect;
            double dy = (1.0 - 2.0 * (y + 0.5) / h) * tan_half;
            double dz = 1.0;
            const double inv = 1.0 / sqrt(dx * dx + dy * dy + dz * dz);
            dx *= inv, dy *= inv, dz *= inv;
            /* |o + t d|^2 = 1 with o = (0, 0, -5) */
            const double b = -5.0 * dz, c = 25.0 - 1.0;
            const double disc = b * b - c;
            float* p = planes;
            for (int k = 0; k < NUM_PLANES; ++k) p[k * n + i] = 0.0f;
            if (disc < 0.0) {
                coverage[i] = 0;
                p[3 * n + i] = (float)dx, p[4 * n + i] = (float)dy, p[5 * n + i] = (float)dz;
                continue;
            }
            const double t = -b - sqrt(disc);
            const double px = t * dx, py = t * dy, pz = -5.0 + t * dz;
            const double r = sqrt(px * px + py * py + pz * pz);
            coverage[i] = 1;
            p[0 * n + i] = (float)px, p[1 * n + i] = (float)py, p[2 * n + i] = (float)pz;
            p[3 * n + i] = (float)(px / r), p[4 * n + i] = (float)(py / r), p[5 * n + i] = (float)(pz / r);
            p[6 * n + i] = 1.0f, p[7 * n + i] = 0.0f, p[8 * n + i] = 0.0f;         /* red albedo */
            p[9 * n + i] = 0.5f;                                                    /* metallic */
            p[10 * n + i] = (float)((double)x / (w - 1));                           /* roughness */
            p[11 * n + i] = 1.0f;                                                   /* AO (unused) */
        }
    }
}

/* A small procedural sky (R16G16B16A16_UNORM): zenith blue to horizon white, ground gray. */
static void fill_sky(int w, int h, uint16_t* texels) {
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            const double v = (double)y / (h - 1);
            double rgb[3];
            if (v < 0.5) {
                const double s = v / 0.5;
                rgb[0] = 0.25 + 0.75 * s, rgb[1] = 0.45 + 0.55 * s, rgb[2] = 0.9 + 0.1 * s;
            } else {
                rgb[0] = rgb[1] = rgb[2] = 0.35;
            }
            uint16_t* t = texels + 4 * ((size_t)y * w + x);
            for (int k = 0; k < 3; ++k) t[k] = (uint16_t)lrint(rgb[k] * 65535.0);
            t[3] = 65535;
        }
    }
}

static uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

int main(int argc, char** argv) {
    int w = 640, h = 360;
    const char* out_path = "sphere.ppm";
    const char* dump_path = NULL;
    int host_only = 0; /* --host-only: the host half (G-buffer + sky fill) and its checksum, no HIP call */
    for (int a = 1; a < argc; ++a) {
        if (!strcmp(argv[a], "--host-only")) host_only = 1;
        else if (a + 1 >= argc) return 2;
        else if (!strcmp(argv[a], "--width")) w = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--height")) h = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--out")) out_path = argv[++a];
        else if (!strcmp(argv[a], "--dump")) dump_path = argv[++a];
        else return 2;
    }
    if (w < 2 || h < 2) return 2;
    const size_t n = (size_t)w * h;
    const int sky_w = 64, sky_h = 32;

    float* planes = malloc(sizeof(float) * NUM_PLANES * n);
    uint8_t* coverage = malloc(n);
    uint8_t* frame = malloc(4 * n);
    uint16_t* sky = malloc(sizeof(uint16_t) * 4 * sky_w * sky_h);
    if (!planes || !coverage || !frame || !sky) return 1;
    fill_gbuffer(w, h, planes, coverage);
    fill_sky(sky_w, sky_h, sky);
    if (host_only) {
        printf("shade_sphere: %dx%d host G-buffer fnv1a %016llx coverage %016llx sky %016llx\n", w, h,
               (unsigned long long)fnv1a((const uint8_t*)planes, sizeof(float) * NUM_PLANES * n),
               (unsigned long long)fnv1a(coverage, n),
               (unsigned long long)fnv1a((const uint8_t*)sky, sizeof(uint16_t) * 4 * sky_w * sky_h));
        free(planes), free(coverage), free(frame), free(sky);
        return 0;
    }

    /* Device buffers: the caller owns them (the library never frees them). */
    float* d_planes;
    uint8_t *d_cov, *d_frame;
    check_hip(hipMalloc((void**)&d_planes, sizeof(float) * NUM_PLANES * n), "hipMalloc planes");
    check_hip(hipMalloc((void**)&d_cov, n), "hipMalloc coverage");
    check_hip(hipMalloc((void**)&d_frame, 4 * n), "hipMalloc frame");
    check_hip(hipMemcpy(d_planes, planes, sizeof(float) * NUM_PLANES * n, hipMemcpyHostToDevice), "upload planes");
    check_hip(hipMemcpy(d_cov, coverage, n, hipMemcpyHostToDevice), "upload coverage");

    pbr_context* ctx = NULL;
    check_pbr(pbr_context_create(0, &ctx), "pbr_context_create", NULL);

    /* UpdateMainPassCB (PBRApp.cpp:455-502): eye, ambient, the four directional lights. */
    pbr_light lights[4];
    memset(lights, 0, sizeof lights);
    const float d = 0.57735f;
    const float dirs[4][3] = {{d, d, d}, {d, -d, d}, {-d, d, d}, {-d, -d, d}};
    for (int i = 0; i < 4; ++i) {
        lights[i].spot_power = 64.0f;
        for (int k = 0; k < 3; ++k) {
            lights[i].strength[k] = 0.25f;
            lights[i].direction[k] = dirs[i][k];
        }
    }
    pbr_pass_desc pass;
    memset(&pass, 0, sizeof pass);
    pass.eye_pos_w[2] = -5.0f;
    for (int k = 0; k < 3; ++k) {
        pass.ambient_light[k] = 0.03f;
        pass.fresnel_r0[k] = 0.04f;
    }
    pass.opacity = 1.0f;
    pass.num_dir_lights = 4;
    pass.ambient_mode = PBR_AMBIENT_CONSTANT;
    pass.lights = lights;
    check_pbr(pbr_set_pass(ctx, &pass, NULL), "pbr_set_pass", ctx);
    check_pbr(pbr_set_sky_map(ctx, sky, sky_w, sky_h, NULL), "pbr_set_sky_map", ctx);

    pbr_gbuffer_soa gb;
    memset(&gb, 0, sizeof gb);
    for (int k = 0; k < 3; ++k) {
        gb.pos_w[k] = d_planes + (0 + k) * n;
        gb.normal_w[k] = d_planes + (3 + k) * n;
        gb.albedo[k] = d_planes + (6 + k) * n;
    }
    gb.metallic = d_planes + 9 * n;
    gb.roughness = d_planes + 10 * n;
    gb.width = w;
    gb.height = h;
    gb.row_stride = w;

    pbr_frame_desc fr;
    memset(&fr, 0, sizeof fr);
    fr.out = d_frame;
    fr.out_row_stride = w;
    fr.format = PBR_OUTPUT_RGBA8_UNORM;
    fr.coverage = d_cov;
    fr.coverage_row_stride = w;
    check_pbr(pbr_shade_frame(ctx, &gb, &fr, NULL), "pbr_shade_frame", ctx);
    check_hip(hipDeviceSynchronize(), "shade");
    check_hip(hipMemcpy(frame, d_frame, 4 * n, hipMemcpyDeviceToHost), "download frame");

    FILE* f = fopen(out_path, "wb");
    if (!f) return 1;
    fprintf(f, "P6\n%d %d\n255\n", w, h);
    for (size_t i = 0; i < n; ++i) fwrite(frame + 4 * i, 1, 3, f);
    fclose(f);
    if (dump_path) {  /* w, h, sky_w, sky_h, planes, coverage, sky texels, frame */
        FILE* g = fopen(dump_path, "wb");
        if (!g) return 1;
        const int32_t dims[4] = {w, h, sky_w, sky_h};
        fwrite(dims, sizeof dims, 1, g);
        fwrite(planes, sizeof(float), NUM_PLANES * n, g);
        fwrite(coverage, 1, n, g);
        fwrite(sky, sizeof(uint16_t), 4 * (size_t)sky_w * sky_h, g);
        fwrite(frame, 1, 4 * n, g);
        fclose(g);
    }
    printf("shade_sphere: %dx%d RGBA8 frame -> %s, fnv1a %016llx\n", w, h, out_path,
           (unsigned long long)fnv1a(frame, 4 * n));

    check_pbr(pbr_context_destroy(ctx), "pbr_context_destroy", NULL);
    (void)hipFree(d_planes);
    (void)hipFree(d_cov);
    (void)hipFree(d_frame);
    free(planes), free(coverage), free(frame), free(sky);
    return 0;
}
