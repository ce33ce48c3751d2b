// pbr_context.hip -- the C ABI of include/pbr/pbr_shade.h: context lifetime, pass/env upload and
// the shade entry point. Host code only; the kernels live in shade_kernels.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <new>
#include <string>

#include "pbr/pbr_shade.h"
#include "shade_kernels.h"
#include "pbr_debug_bounds.h"
#include "pbr_build_info.h"

// The build records of the library's units (pbr_build_info.h). Weak: a profiling build compiles the balanced kernels
// into shade_kernels.hip's unit, so shade_kernels_bal's record is then absent (null) and not listed.
extern "C" {
extern const char pbr_unit_info_shade_kernels[] __attribute__((weak));
extern const char pbr_unit_info_shade_kernels_bal[] __attribute__((weak));
extern const char pbr_unit_info_gbuffer_fill[] __attribute__((weak));
__attribute__((used)) const char pbr_unit_info_pbr_context[] =
    PBR_UNIT_INFO("pbr_context", PBR_BI_SWITCH(PBR_DEBUG_BOUNDS));
}

// Cross-stream ordering of the context's device resources (the reference's 3-deep FrameResource ring,
// FrameResource.h:111-140, PBRApp.cpp:220-243, is the same idea on D3D12 fences). A resource -- a light slot,
// the env map, the sky map -- remembers which streams have queued a pass reading it since it was last written
// and which stream wrote it (with an event after the write):
//   * before it is overwritten on stream w, w waits (stream-side, no host synchronisation) for the last pass of
//     every other stream that read it -- each stream's `last_pass` event, recorded after its launches;
//     waiting for a later pass of that stream is merely early;
//   * a pass on stream s that reads it waits for the write's event once, unless s wrote it.
// A context used from one stream records nothing per launch (every reader is the writer's stream). The first
// launch on a second stream synchronises the device once, so the earlier single-stream passes are complete and
// need no event; from then on each launch records its stream's last_pass.
struct StreamState {
    hipStream_t stream = nullptr;
    hipEvent_t last_pass = nullptr;  // multi-stream contexts: recorded after every launch on `stream`
    // Statistics of the last pass on this stream: one record of pbr::kStatsPerBlock int32 per statistics slot
    // (one per wave in the pair layout, per workgroup in the one-pixel layout; pbr::StatField), summed on the
    // host by pbr_last_pass_stats / pbr_last_cull_stats. Written only by this stream's passes, so a pass never
    // overwrites the record of a pass on another stream.
    int32_t* d_stats = nullptr;
    int64_t stats_capacity = 0;  // slots
    int64_t tiles = 0, slots = 0;
    bool culled = false;
    std::string kernel;  // the last pass's kernel (pbr_last_pass_kernel)
};

struct Resource {
    std::vector<int> readers;  // StreamState indices that launched a pass reading it since the last write
    int writer = -1;           // StreamState index of the stream that wrote it last (-1: none / host-complete)
    hipEvent_t written = nullptr;  // recorded on the writer's stream after the write
};

struct pbr_context {
    int device = 0;
    std::vector<StreamState> streams;
    // Lights: a ring of device slots (3 float4 per light), each fed from its own pinned staging copy so a host
    // pass struct can be reused as soon as pbr_set_pass returns. Every pbr_set_pass takes the next slot; a
    // launch reads the slot of the pass it was queued with, so setting frame k+1's pass (on any stream) never
    // overwrites the lights a queued frame k reads.
    static constexpr int kSlots = 4;
    struct LightSlot {
        float4* d = nullptr;
        int capacity = 0;
        pbr_light* h = nullptr;        // pinned staging, PBR_MAX_LIGHTS records
        hipEvent_t copied = nullptr;   // the staging -> device copy
        bool copy_pending = false;
        Resource use;
    };
    LightSlot slots[kSlots];
    int cur_slot = -1;
    int next_slot = 0;
    // Textures: the environment (IBL, g_SkyArray[1]) and the sky (g_SkyArray[0]), each kept as fp32
    // RGBA on the device (decoded once from R16G16B16A16_UNORM, or uploaded as fp32).
    struct Texture {
        uint16_t* d_u16 = nullptr;  // UNORM16 upload staging
        float4* d = nullptr;
        int w = 0, h = 0, capacity = 0;
        bool nonneg = true;  // no negative or NaN texel (PBR_FLAG_FAITHFUL precondition for the IBL)
        Resource use;
    };
    Texture env, sky;
    // Current pass.
    pbr::PassArgs pass{};
    int ambient_mode = 0;
    uint32_t flags = 0;
    bool pass_set = false;
    bool faithful_pass_ok = false;  // light strengths and the constant ambient are finite and >= 0
    bool faithful_count_terms = false;  // > 64 lights (culled pass): the kernel counts summed terms per wave
    int last_stream = -1;  // StreamState index of the context's last pass (pbr_last_pass_stats fallback)
    // Wave-balanced point-light lists (pbr_balanced.h) for untiled passes with at least this many point lights
    // and no spot lights; -1: the measured crossover of the mode (kBalancedMinFaithful / kBalancedMinExact);
    // PBR_BALANCED_MIN overrides both (0 disables).
    int balanced_min = -1;
    bool points_flag_ok = false;  // pbr_set_pass: every point light inside the fast-path window
    bool points_quarter_ok = false;  // ... and every point strength within 2^50 (the exact balanced items' 4x radiance)
    int pixels_per_thread = 2;  // kernel layout: packed pixel pairs (measured faster); PBR_PIXELS_PER_THREAD=1 overrides
    bool lean = true;  // uniform-loop passes without a sky pass use the lean pair kernel (PBR_LEAN=0: off)
    std::string last_error;
    std::mutex mu;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int fail_hip(pbr_context* ctx, hipError_t e, const char* what, int status = PBR_ERR_HIP) {
    if (ctx) {
        ctx->last_error = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    }
    return e == hipErrorOutOfMemory ? PBR_ERR_OUT_OF_MEMORY : status;
}

bool is_ambient_mode(int m) { return m == PBR_AMBIENT_CONSTANT || m == PBR_AMBIENT_IBL_DIFFUSE; }

void forget_readers(pbr_context* ctx);

// PBR_DEBUG_BOUNDS builds (pbr_debug_bounds.h): one bounds-flag buffer per device, allocated, cleared and published
// to the kernels by the first context created on it; product builds have none.
constexpr int kBoundsMaxDevices = 64;
constexpr size_t kBoundsBytes = sizeof(uint32_t) * 2 * pbr::kBoundsClasses;
std::mutex g_bounds_mu;
uint32_t* g_bounds_buf[kBoundsMaxDevices] = {};

hipError_t arm_bounds(int dev) {  // current device = dev
    if (!PBR_DEBUG_BOUNDS) return hipSuccess;
    if (dev < 0 || dev >= kBoundsMaxDevices) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_bounds_mu);
    if (g_bounds_buf[dev]) return hipSuccess;
    uint32_t* b = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&b), kBoundsBytes);
    if (e == hipSuccess) e = hipMemset(b, 0, kBoundsBytes);
    if (e == hipSuccess) e = pbr::debug_bounds_publish(b);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess)
        g_bounds_buf[dev] = b;
    else if (b)
        (void)hipFree(b);
    return e;
}

// PBR_DEBUG_BOUNDS_SKEW=1 (bounds-checked builds): the output extent the checks use is one column narrower than
// the frame, so every pass must report class 1 -- the negative control of tests/test_gpu_debug_bounds.py.
bool debug_bounds_skew() {
    static const bool skew = [] {
        const char* e = std::getenv("PBR_DEBUG_BOUNDS_SKEW");
        return PBR_DEBUG_BOUNDS && e != nullptr && std::atoi(e) != 0;
    }();
    return skew;
}

// Streams a context tracks at once. Contexts expect a small, long-lived set of streams (a FrameResource-style
// ring); a caller that keeps creating new ones pays one device synchronisation per new stream, and past this
// bound the table is pruned at that synchronisation, so it never grows without limit.
constexpr size_t kMaxStreams = 16;

// The StreamState of `s` (created on first use). Caller holds ctx->mu and the device guard. A new stream
// beside existing ones: the device is synchronised once, so every pass queued so far is complete and no
// resource has a pending reader (the single-stream passes recorded no event). A full table is pruned then to the
// context's last pass stream (whose statistics pbr_last_pass_stats falls back to): the others' records go, which
// is safe as nothing of theirs is in flight. A destroyed stream whose handle value a new stream reuses is taken for
// the old one; the contract (pbr_shade.h) asks callers to let a stream's passes finish before destroying it.
int stream_index(pbr_context* ctx, hipStream_t s, hipError_t& e) {
    for (size_t i = 0; i < ctx->streams.size(); ++i)
        if (ctx->streams[i].stream == s) return (int)i;
    if (!ctx->streams.empty()) {
        e = hipDeviceSynchronize();
        if (e != hipSuccess) return -1;
        forget_readers(ctx);
        if (ctx->streams.size() >= kMaxStreams) {
            std::vector<StreamState> keep;
            for (size_t i = 0; i < ctx->streams.size(); ++i) {
                StreamState& st = ctx->streams[i];
                if ((int)i == ctx->last_stream) {
                    keep.push_back(std::move(st));
                    continue;
                }
                if (st.last_pass) (void)hipEventDestroy(st.last_pass);
                if (st.d_stats) (void)hipFree(st.d_stats);
            }
            ctx->last_stream = keep.empty() ? -1 : 0;
            ctx->streams = std::move(keep);
        }
    }
    StreamState st;
    st.stream = s;
    // device-scope release: only other streams of this device (and host waits before a free) observe it
    e = hipEventCreateWithFlags(&st.last_pass, hipEventDisableTiming | hipEventReleaseToDevice);
    if (e != hipSuccess) return -1;
    ctx->streams.push_back(st);
    return (int)ctx->streams.size() - 1;
}

// Order a write of `r` on stream `w` (index wi) after every pass of another stream that read it.
hipError_t before_write(pbr_context* ctx, Resource& r, hipStream_t w, int wi) {
    for (int i : r.readers) {
        if (i == wi) continue;  // same stream: already ordered
        const hipError_t e = hipStreamWaitEvent(w, ctx->streams[i].last_pass, 0);
        if (e != hipSuccess) return e;
    }
    r.readers.clear();
    return hipSuccess;
}

// Release the memory `p` of resource `r`, which is growing, in stream order on `w` (index wi): `w` waits (stream-side)
// for the last pass of every other stream that read `r` and for a write of `r` queued on another stream, then the
// memory goes back to the device's pool with hipFreeAsync. Nothing blocks the host or an unrelated stream, and the
// sequence is legal inside a graph capture of `w`. A context used from one stream has every reader on `w` itself (a
// second stream's first launch synchronises the device and clears the records, stream_index), so stream order alone
// covers them; a multi-stream context records each stream's `last_pass` after every launch. Those events outlive the
// caller's stream handles, so a reader stream destroyed after its passes finished (the contract, pbr_shade.h) is never
// touched. The resources are allocated with hipMallocAsync on the writing stream for the same reason.
hipError_t free_after_readers(pbr_context* ctx, Resource& r, void* p, hipStream_t w, int wi) {
    hipError_t e = before_write(ctx, r, w, wi);
    if (e == hipSuccess && r.writer >= 0 && r.writer != wi) e = hipStreamWaitEvent(w, r.written, 0);
    if (e == hipSuccess && p) e = hipFreeAsync(p, w);
    return e;
}

// Record the write of `r` on stream `w` (index wi).
hipError_t after_write(Resource& r, hipStream_t w, int wi) {
    if (!r.written) {
        const hipError_t e = hipEventCreateWithFlags(&r.written, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    r.writer = wi;
    return hipEventRecord(r.written, w);
}

// A pass on stream `s` (index si) is about to read `r`: order it after the write, once per stream.
hipError_t before_read(Resource& r, hipStream_t s, int si) {
    for (int i : r.readers)
        if (i == si) return hipSuccess;
    if (r.writer >= 0 && r.writer != si) {
        const hipError_t e = hipStreamWaitEvent(s, r.written, 0);
        if (e != hipSuccess) return e;
    }
    r.readers.push_back(si);
    return hipSuccess;
}

// After a device synchronisation: every queued read and write of the context's resources is complete.
void forget_readers(pbr_context* ctx) {
    for (pbr_context::LightSlot& sl : ctx->slots) {
        sl.use.readers.clear();
        sl.use.writer = -1;
    }
    for (pbr_context::Texture* t : {&ctx->env, &ctx->sky}) {
        t->use.readers.clear();
        t->use.writer = -1;
    }
}

}  // namespace

extern "C" {

int pbr_abi_version(void) { return PBR_ABI_VERSION; }

const char* pbr_build_info(void) {
    static const std::string info = [] {
        std::string r = "{\"abi\": " + std::to_string(PBR_ABI_VERSION) + ", \"units\": [";
        bool first = true;
        for (const char* u : {pbr_unit_info_pbr_context, pbr_unit_info_shade_kernels, pbr_unit_info_shade_kernels_bal,
                              pbr_unit_info_gbuffer_fill}) {
            if (u == nullptr) continue;
            r += first ? "" : ", ";
            r += u;
            first = false;
        }
        return r + "]}";
    }();
    return info.c_str();
}

const char* pbr_strerror(int status) {
    switch (status) {
        case PBR_OK: return "ok";
        case PBR_ERR_INVALID_ARGUMENT: return "invalid argument";
        case PBR_ERR_NO_DEVICE: return "no HIP device";
        case PBR_ERR_OUT_OF_MEMORY: return "out of device memory";
        case PBR_ERR_LAUNCH: return "kernel launch failed";
        case PBR_ERR_HIP: return "HIP runtime error";
        case PBR_ERR_NOT_READY: return "pass or environment map not set";
        case PBR_ERR_UNSUPPORTED: return "unsupported";
        default: return "unknown status";
    }
}

const char* pbr_last_error(const pbr_context* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int pbr_context_create(int device, pbr_context** out_ctx) {
    if (!out_ctx) return PBR_ERR_INVALID_ARGUMENT;
    *out_ctx = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return PBR_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return PBR_ERR_INVALID_ARGUMENT;
    pbr_context* ctx = new (std::nothrow) pbr_context();
    if (!ctx) return PBR_ERR_OUT_OF_MEMORY;
    ctx->device = device;
    if (const char* e = std::getenv("PBR_PIXELS_PER_THREAD")) ctx->pixels_per_thread = std::atoi(e) == 1 ? 1 : 2;
    if (const char* e = std::getenv("PBR_BALANCED_MIN")) ctx->balanced_min = std::atoi(e);
    if (const char* e = std::getenv("PBR_LEAN")) ctx->lean = std::atoi(e) != 0;
    DeviceGuard g(device);
    if (!g.ok) {
        delete ctx;
        return PBR_ERR_NO_DEVICE;
    }
    hipError_t e = arm_bounds(device);
    for (int i = 0; e == hipSuccess && i < pbr_context::kSlots; ++i) {
        e = hipHostMalloc(reinterpret_cast<void**>(&ctx->slots[i].h), sizeof(pbr_light) * PBR_MAX_LIGHTS,
                          hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->slots[i].copied, hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        pbr_context_destroy(ctx);
        return e == hipErrorOutOfMemory ? PBR_ERR_OUT_OF_MEMORY : PBR_ERR_HIP;
    }
    *out_ctx = ctx;
    return PBR_OK;
}

int pbr_context_destroy(pbr_context* ctx) {
    if (!ctx) return PBR_ERR_INVALID_ARGUMENT;
    {
        DeviceGuard g(ctx->device);
        (void)hipDeviceSynchronize();
        // Light slots and textures come from the stream-ordered pool (hipMallocAsync): returned the same way, after
        // the synchronisation above, and the pool's frees completed by the one below.
        for (pbr_context::LightSlot& sl : ctx->slots) {
            if (sl.copied) (void)hipEventDestroy(sl.copied);
            if (sl.h) (void)hipHostFree(sl.h);
            if (sl.d) (void)hipFreeAsync(sl.d, nullptr);
            if (sl.use.written) (void)hipEventDestroy(sl.use.written);
        }
        for (pbr_context::Texture* t : {&ctx->env, &ctx->sky}) {
            if (t->d_u16) (void)hipFreeAsync(t->d_u16, nullptr);
            if (t->d) (void)hipFreeAsync(t->d, nullptr);
            if (t->use.written) (void)hipEventDestroy(t->use.written);
        }
        for (StreamState& st : ctx->streams) {
            if (st.last_pass) (void)hipEventDestroy(st.last_pass);
            if (st.d_stats) (void)hipFree(st.d_stats);
        }
        (void)hipDeviceSynchronize();
    }
    delete ctx;
    return PBR_OK;
}

int pbr_set_pass(pbr_context* ctx, const pbr_pass_desc* pass, void* stream) {
    if (!ctx || !pass) return PBR_ERR_INVALID_ARGUMENT;
    const int nd = pass->num_dir_lights, np = pass->num_point_lights, ns = pass->num_spot_lights;
    if (nd < 0 || np < 0 || ns < 0) return PBR_ERR_INVALID_ARGUMENT;
    const long long n = (long long)nd + np + ns;
    if (n > PBR_MAX_LIGHTS) return PBR_ERR_INVALID_ARGUMENT;
    if (n > 0 && !pass->lights) return PBR_ERR_INVALID_ARGUMENT;
    if (!is_ambient_mode(pass->ambient_mode)) return PBR_ERR_INVALID_ARGUMENT;
    const uint32_t known =
        PBR_FLAG_F0_PLANE | PBR_FLAG_APPLY_AO | PBR_FLAG_TILED_CULLING | PBR_FLAG_EXACT_ONLY | PBR_FLAG_FAITHFUL |
        PBR_FLAG_ALPHA_TEST;
    if (pass->flags & ~known) return PBR_ERR_INVALID_ARGUMENT;

    std::lock_guard<std::mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok) return PBR_ERR_NO_DEVICE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipSuccess;
    const int si = stream_index(ctx, s, e);
    if (si < 0) return fail_hip(ctx, e, "pbr_set_pass stream");
    // The next slot of the ring: its staging copy must have left the host buffer, and its device copy is
    // overwritten only after the queued passes that read it (stream-side waits, before_write).
    const int slot = ctx->next_slot;
    pbr_context::LightSlot& sl = ctx->slots[slot];
    if (sl.copy_pending) {
        e = hipEventSynchronize(sl.copied);
        if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass staging wait");
        sl.copy_pending = false;
    }
    if (n > sl.capacity) {
        // Growing: the old buffer may still be read by queued passes (released after them, in stream order).
        if (sl.d) {
            e = free_after_readers(ctx, sl.use, sl.d, s, si);
            if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass slot release");
            sl.d = nullptr;
            sl.capacity = 0;
        }
        int cap = 64;
        while (cap < n) cap *= 2;
        e = hipMallocAsync(reinterpret_cast<void**>(&sl.d), sizeof(pbr_light) * (size_t)cap, s);
        if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass hipMalloc");
        sl.capacity = cap;
    }
    bool points_ok = true;  // every point light's fast-path flag is set (the balanced pass needs it)
    // The exact balanced kernel's items carry 4x the radiance (pbr_balanced.h, stage_balanced_lights; brdf_x2's QUARTER
    // form): with |strength| <= 2^50 the scaled products stay below 2^126 (term factors <= 2^57.1 x 2^13.3 attenuation
    // x 4 x 2^50), so every scaling is exact and no term overflows where the reference's does not.
    bool quarter_ok = true;
    if (n > 0) {
        std::memcpy(sl.h, pass->lights, sizeof(pbr_light) * (size_t)n);
        // The kernel's per-light fast-path flag travels in the unused pad1 of the uploaded copy
        // (the caller's array is not touched): directional L = -Direction components, point / spot
        // positions, each 0 or |x| in [2^-20, 16] / [2^-20, 2^20] (pbr_device_math.h, light_window_ok),
        // and a finite point / spot strength.
        for (long long i = 0; i < n; ++i) {
            pbr_light& L = sl.h[i];
            const bool directional = i < nd;
            const float* c = directional ? L.direction : L.position;
            const float hi = directional ? 16.0f : 0x1p20f;
            bool ok = true;
            for (int k = 0; k < 3; ++k) {
                const float a = std::fabs(c[k]);
                ok = ok && (a == 0.0f || (a >= 0x1p-20f && a <= hi));
                // point / spot: a finite strength, so that an out-of-range lane's zero-attenuated
                // contribution is +-0 (pbr_device_math_x2.h, point_or_spot_x2)
                if (!directional) ok = ok && std::isfinite(L.strength[k]);
            }
            L.pad1 = ok ? 1.0f : 0.0f;
            if (i >= nd && i < nd + np) {
                points_ok = points_ok && ok;
                for (int k = 0; k < 3; ++k) quarter_ok = quarter_ok && std::fabs(L.strength[k]) <= 0x1p50f;
            }
        }
        e = before_write(ctx, sl.use, s, si);
        if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass order");
        e = hipMemcpyAsync(sl.d, sl.h, sizeof(pbr_light) * (size_t)n, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass copy");
        e = hipEventRecord(sl.copied, s);
        if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass record");
        sl.copy_pending = true;
        e = after_write(sl.use, s, si);
        if (e != hipSuccess) return fail_hip(ctx, e, "pbr_set_pass record");
    }
    ctx->cur_slot = slot;
    ctx->next_slot = (slot + 1) % pbr_context::kSlots;
    pbr::PassArgs& p = ctx->pass;
    for (int i = 0; i < 3; ++i) {
        p.eye[i] = pass->eye_pos_w[i];
        p.ambient[i] = pass->ambient_light[i];
        p.fresnel_r0[i] = pass->fresnel_r0[i];
    }
    p.opacity = pass->opacity;
    p.eye_ok = 1;
    for (int i = 0; i < 3; ++i) {  // the fast-path window of the (uniform) eye: 0 or |x| in [2^-20, 2^20]
        const float a = std::fabs(pass->eye_pos_w[i]);
        if (!(a == 0.0f || (a >= 0x1p-20f && a <= 0x1p20f))) p.eye_ok = 0;
    }
    p.n_dir = nd;
    p.n_point = np;
    p.n_spot = ns;
    // PBR_FLAG_FAITHFUL's error bound needs every term of the light sum >= 0
    // (pbr_device_math_x2.h, brdf_faithful_x2): finite non-negative strengths and a non-negative constant
    // ambient; and at most 64 summed terms, since the sum's rounding drift grows by <= 1 ulp per term --
    // with tiled culling the kernel counts each wave's surviving lights (faithful mode 2).
    ctx->faithful_count_terms = n > 64;
    bool nonneg = n <= 64 || (pass->flags & PBR_FLAG_TILED_CULLING) != 0;
    for (long long i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) nonneg = nonneg && std::isfinite(pass->lights[i].strength[k]) && pass->lights[i].strength[k] >= 0.0f;
    if (pass->ambient_mode == PBR_AMBIENT_CONSTANT)
        for (int k = 0; k < 3; ++k) nonneg = nonneg && pass->ambient_light[k] >= 0.0f;
    ctx->faithful_pass_ok = nonneg;
    ctx->points_flag_ok = points_ok;
    ctx->points_quarter_ok = points_ok && quarter_ok;
    ctx->ambient_mode = pass->ambient_mode;
    ctx->flags = pass->flags;
    ctx->pass_set = true;
    return PBR_OK;
}

}  // extern "C"

namespace {

// Upload a width x height RGBA texture (UNORM16 -> decoded on the device, or fp32 as given) into slot
// `t`. Synchronous with respect to the host buffer: it may be released on return.
int set_texture(pbr_context* ctx, pbr_context::Texture& t, const void* texels, bool unorm16, int32_t width,
                int32_t height, void* stream, const char* what) {
    if (!ctx || !texels || width <= 0 || height <= 0) return PBR_ERR_INVALID_ARGUMENT;
    if ((long long)width * height > (1ll << 26)) return PBR_ERR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok) return PBR_ERR_NO_DEVICE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int n = width * height;
    hipError_t e = hipSuccess;
    const int si = stream_index(ctx, s, e);
    if (si < 0) return fail_hip(ctx, e, what);
    if (n > t.capacity) {
        // Growing: the old texture may still be read by queued passes (released after them, in stream order).
        e = free_after_readers(ctx, t.use, t.d_u16, s, si);
        if (e == hipSuccess && t.d) e = hipFreeAsync(t.d, s);
        if (e != hipSuccess) return fail_hip(ctx, e, what);
        t.d_u16 = nullptr;
        t.d = nullptr;
        t.capacity = 0;
        e = hipMallocAsync(reinterpret_cast<void**>(&t.d_u16), sizeof(uint16_t) * 4 * (size_t)n, s);
        if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&t.d), sizeof(float4) * (size_t)n, s);
        if (e != hipSuccess) return fail_hip(ctx, e, what);
        t.capacity = n;
    }
    // Replaced in place: after the queued passes (of any stream) that read the old texels.
    e = before_write(ctx, t.use, s, si);
    if (e != hipSuccess) return fail_hip(ctx, e, what);
    if (unorm16) {
        e = hipMemcpyAsync(t.d_u16, texels, sizeof(uint16_t) * 4 * (size_t)n, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return fail_hip(ctx, e, what);
        e = pbr::launch_decode_unorm16(t.d_u16, t.d, n, s);
        if (e != hipSuccess) return fail_hip(ctx, e, "decode_unorm16_kernel", PBR_ERR_LAUNCH);
    } else {
        e = hipMemcpyAsync(t.d, texels, sizeof(float4) * (size_t)n, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return fail_hip(ctx, e, what);
    }
    e = hipStreamSynchronize(s);  // the (pageable) host texels may be released on return
    if (e != hipSuccess) return fail_hip(ctx, e, what);
    t.use.writer = -1;  // complete: later passes on any stream see the new texels
    t.w = width;
    t.h = height;
    t.nonneg = true;
    if (!unorm16) {
        const float* f = static_cast<const float*>(texels);
        for (size_t i = 0; i < 4 * (size_t)n && t.nonneg; ++i) t.nonneg = f[i] >= 0.0f;  // false for NaN
    }
    return PBR_OK;
}

bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

int shade(pbr_context* ctx, const pbr_gbuffer_soa* gb, const pbr_frame_desc* fr, void* stream) {
    if (!ctx || !gb || !fr) return PBR_ERR_INVALID_ARGUMENT;
    if (gb->width < 0 || gb->height < 0 || gb->row_stride < gb->width || fr->out_row_stride < gb->width)
        return PBR_ERR_INVALID_ARGUMENT;
    if (fr->format != PBR_OUTPUT_RGBA32F && fr->format != PBR_OUTPUT_RGBA8_UNORM) return PBR_ERR_INVALID_ARGUMENT;
    if (fr->coverage && fr->coverage_row_stride < gb->width) return PBR_ERR_INVALID_ARGUMENT;
    // Everything below reads context state that pbr_set_pass / pbr_set_*_map write under the same
    // mutex: the launch arguments are built (and the kernel queued) in one critical section, so a
    // concurrent set_pass can never tear them.
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->pass_set) return PBR_ERR_NOT_READY;
    if (gb->width == 0 || gb->height == 0) return PBR_OK;  // empty frame: nothing is read or written
    if (!fr->out) return PBR_ERR_INVALID_ARGUMENT;
    if (!aligned(fr->out, fr->format == PBR_OUTPUT_RGBA8_UNORM ? 4 : 16)) return PBR_ERR_INVALID_ARGUMENT;
    const bool f0_plane = (ctx->flags & PBR_FLAG_F0_PLANE) != 0;
    const bool apply_ao = (ctx->flags & PBR_FLAG_APPLY_AO) != 0;
    const bool cull = (ctx->flags & PBR_FLAG_TILED_CULLING) != 0;
    for (int i = 0; i < 3; ++i)
        if (!gb->pos_w[i] || !gb->normal_w[i] || !gb->albedo[i]) return PBR_ERR_INVALID_ARGUMENT;
    if (!gb->metallic || !gb->roughness) return PBR_ERR_INVALID_ARGUMENT;
    if (apply_ao && !gb->ao) return PBR_ERR_INVALID_ARGUMENT;
    if (f0_plane && (!gb->f0[0] || !gb->f0[1] || !gb->f0[2])) return PBR_ERR_INVALID_ARGUMENT;
    const bool alpha_test = (ctx->flags & PBR_FLAG_ALPHA_TEST) != 0;
    if (alpha_test && !gb->opacity) return PBR_ERR_INVALID_ARGUMENT;
    if (ctx->ambient_mode == PBR_AMBIENT_IBL_DIFFUSE && !ctx->env.d) return PBR_ERR_NOT_READY;
    if (fr->coverage && !ctx->sky.d) return PBR_ERR_NOT_READY;  // background pixels need the sky map

    pbr::LaunchArgs a{};
    const float* planes[15] = {gb->pos_w[0], gb->pos_w[1], gb->pos_w[2], gb->normal_w[0], gb->normal_w[1],
                               gb->normal_w[2], gb->albedo[0], gb->albedo[1], gb->albedo[2], gb->metallic,
                               gb->roughness, gb->ao, gb->f0[0], gb->f0[1], gb->f0[2]};
    for (int i = 0; i < 15; ++i) a.gb.plane[i] = planes[i] ? planes[i] : planes[0];
    a.gb.plane[15] = alpha_test ? gb->opacity : planes[0];
    a.gb.alpha_test = alpha_test;
    a.gb.width = gb->width;
    a.gb.height = gb->height;
    a.gb.row_stride = gb->row_stride;
    a.gb.pairs_aligned = (gb->row_stride % 2) == 0;
    for (int i = 0; i < 16; ++i)
        if (!aligned(a.gb.plane[i], 8)) a.gb.pairs_aligned = false;
    a.ps = ctx->pass;
    a.ps.env_w = ctx->env.w;
    a.ps.env_h = ctx->env.h;
    a.ps.sky_w = ctx->sky.w;
    a.ps.sky_h = ctx->sky.h;
    a.lights = ctx->cur_slot >= 0 ? ctx->slots[ctx->cur_slot].d : nullptr;
    a.env = ctx->env.d;
    a.frame.out = fr->out;
    a.frame.out_stride = fr->out_row_stride;
    a.frame.format = fr->format == PBR_OUTPUT_RGBA8_UNORM ? pbr::kOutRgba8 : pbr::kOutRgba32f;
    a.frame.coverage = fr->coverage;
    a.frame.coverage_stride = fr->coverage_row_stride;
    a.frame.sky = ctx->sky.d;
    a.frame.width = gb->width - (debug_bounds_skew() ? 1 : 0);
    a.frame.height = gb->height;
    a.ambient_mode = ctx->ambient_mode;
    a.f0_plane = f0_plane;
    a.apply_ao = apply_ao;
    a.cull = cull;
    a.exact_only = (ctx->flags & PBR_FLAG_EXACT_ONLY) != 0;
    a.ps.faithful = (ctx->flags & PBR_FLAG_FAITHFUL) && !a.exact_only && ctx->faithful_pass_ok &&
                    (ctx->ambient_mode != PBR_AMBIENT_IBL_DIFFUSE || ctx->env.nonneg);
    if (a.ps.faithful && ctx->faithful_count_terms) a.ps.faithful = 2;
    a.pixels_per_thread = ctx->pixels_per_thread;
    // Wave-balanced point-light lists: untiled pair-kernel passes with no spot lights, every point light inside
    // the fast-path window; faithful (1) or exact (2, and no directional lights either) -- the exact variant
    // keeps the reference's order per pixel (bit-identical), the faithful one re-associates.
    // Point-light count from which the balanced lists win (same-box sweeps, 1080p and 4K): the
    // faithful loop between 20 (uniform faster) and 24 lights, the exact loop between 16 and 20.
    constexpr int kBalancedMinFaithful = 22, kBalancedMinExact = 18;
    const int bal_min = ctx->balanced_min >= 0 ? ctx->balanced_min
                        : a.ps.faithful == 1   ? kBalancedMinFaithful
                                               : kBalancedMinExact;
    const bool bal_ok = !cull && a.pixels_per_thread == 2 && bal_min > 0 && ctx->points_flag_ok &&
                        a.ps.n_spot == 0 && a.ps.n_point >= bal_min && a.ps.n_point <= pbr::kBalMaxLights;
    a.ps.balanced = !bal_ok                                                ? 0
                    : a.ps.faithful == 1                                   ? 1
                    : a.ps.faithful == 0 && !a.exact_only && a.ps.n_dir == 0 && ctx->points_quarter_ok ? 2
                                                                           : 0;

    DeviceGuard g(ctx->device);
    if (!g.ok) return PBR_ERR_NO_DEVICE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipSuccess;
    const int si = stream_index(ctx, s, e);
    if (si < 0) return fail_hip(ctx, e, "shade stream");
    StreamState& st = ctx->streams[si];
    {
        const int64_t tiles = pbr::shade_tile_count(gb->width, gb->height, a.pixels_per_thread);
        const int64_t slots = tiles * pbr::shade_stat_slots_per_tile(a.pixels_per_thread);
        if (slots > st.stats_capacity) {
            // Growing: only this stream's passes write the buffer (stream order covers them).
            if (st.d_stats) {
                e = hipStreamSynchronize(s);
                if (e != hipSuccess) return fail_hip(ctx, e, "pass stats sync");
                (void)hipFree(st.d_stats);
                st.d_stats = nullptr;
                st.stats_capacity = 0;
            }
            e = hipMalloc(&st.d_stats, pbr::kStatsPerBlock * sizeof(int32_t) * (size_t)slots);
            if (e != hipSuccess) return fail_hip(ctx, e, "pass stats hipMalloc");
            st.stats_capacity = slots;
        }
        st.tiles = tiles;
        st.slots = slots;
        st.culled = cull;
        a.tile_kept = st.d_stats;
        // The lean pair kernel: uniform light loops (no balanced lists), no sky pass, the fast paths enabled.
        a.lean = ctx->lean && a.pixels_per_thread == 2 && a.ps.balanced == 0 && !fr->coverage && !a.exact_only;
    }
    // Order the pass after the writes of what it reads (lights, textures) made on other streams.
    const bool reads_lights = ctx->cur_slot >= 0 && a.ps.n_dir + a.ps.n_point + a.ps.n_spot > 0;
    if (reads_lights) e = before_read(ctx->slots[ctx->cur_slot].use, s, si);
    if (e == hipSuccess && ctx->ambient_mode == PBR_AMBIENT_IBL_DIFFUSE) e = before_read(ctx->env.use, s, si);
    if (e == hipSuccess && fr->coverage) e = before_read(ctx->sky.use, s, si);
    if (e != hipSuccess) return fail_hip(ctx, e, "shade order");
    e = pbr::launch_shade(a, s);
    if (e != hipSuccess) return fail_hip(ctx, e, "shade_tile_kernel launch", PBR_ERR_LAUNCH);
    st.kernel = pbr::launched_kernel(a);
    if (ctx->streams.size() > 1) {
        e = hipEventRecord(st.last_pass, s);
        if (e != hipSuccess) return fail_hip(ctx, e, "shade record");
    }
    ctx->last_stream = si;
    return PBR_OK;
}

}  // namespace

extern "C" {

int pbr_set_env_map(pbr_context* ctx, const uint16_t* texels, int32_t width, int32_t height, void* stream) {
    return ctx ? set_texture(ctx, ctx->env, texels, true, width, height, stream, "pbr_set_env_map")
               : PBR_ERR_INVALID_ARGUMENT;
}

int pbr_set_env_map_f32(pbr_context* ctx, const float* texels, int32_t width, int32_t height, void* stream) {
    return ctx ? set_texture(ctx, ctx->env, texels, false, width, height, stream, "pbr_set_env_map_f32")
               : PBR_ERR_INVALID_ARGUMENT;
}

int pbr_set_sky_map(pbr_context* ctx, const uint16_t* texels, int32_t width, int32_t height, void* stream) {
    return ctx ? set_texture(ctx, ctx->sky, texels, true, width, height, stream, "pbr_set_sky_map")
               : PBR_ERR_INVALID_ARGUMENT;
}

int pbr_set_sky_map_f32(pbr_context* ctx, const float* texels, int32_t width, int32_t height, void* stream) {
    return ctx ? set_texture(ctx, ctx->sky, texels, false, width, height, stream, "pbr_set_sky_map_f32")
               : PBR_ERR_INVALID_ARGUMENT;
}

int pbr_shade_gbuffer(pbr_context* ctx, const pbr_gbuffer_soa* gb, float* out_rgba, int64_t out_row_stride,
                      void* stream) {
    pbr_frame_desc fr{};
    fr.out = out_rgba;
    fr.out_row_stride = out_row_stride;
    fr.format = PBR_OUTPUT_RGBA32F;
    return shade(ctx, gb, &fr, stream);
}

int pbr_shade_frame(pbr_context* ctx, const pbr_gbuffer_soa* gb, const pbr_frame_desc* frame, void* stream) {
    return shade(ctx, gb, frame, stream);
}

}  // extern "C"

namespace {

// Sum the statistics records of the last pass on `stream` (or, if the context never launched on that stream,
// of its last pass on any stream: the caller's stream is then ordered after it by contract).
int sum_pass_stats(pbr_context* ctx, pbr_pass_stats* out, void* stream, const char* what) {
    *out = pbr_pass_stats{};
    DeviceGuard g(ctx->device);
    if (!g.ok) return PBR_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int si = -1;
    for (size_t i = 0; i < ctx->streams.size(); ++i)
        if (ctx->streams[i].stream == s && ctx->streams[i].tiles > 0) si = (int)i;
    if (si < 0) si = ctx->last_stream;
    if (si < 0 || ctx->streams[si].tiles == 0) return PBR_OK;  // no pass yet (or an empty frame)
    const StreamState& st = ctx->streams[si];
    std::vector<int32_t> h(pbr::kStatsPerBlock * (size_t)st.slots);
    hipError_t e = hipMemcpyAsync(h.data(), st.d_stats, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail_hip(ctx, e, what);
    out->workgroups = st.tiles;
    out->culled = st.culled ? 1 : 0;
    for (size_t t = 0; t < h.size(); t += pbr::kStatsPerBlock) {
        out->cull_tile_lights += h[t + pbr::kStatCullKept];
        out->cull_tiles += h[t + pbr::kStatCullTiles];
        out->exact_pixels += h[t + pbr::kStatExactPixels];
        out->light_terms += h[t + pbr::kStatLightTerms];
        out->geometry_pixels += h[t + pbr::kStatGeometryPixels];
        out->backface_tests += h[t + pbr::kStatBackfaceTests];
    }
    return PBR_OK;
}

}  // namespace

extern "C" {

int pbr_last_cull_stats(pbr_context* ctx, int64_t* sum_tile_lights, int64_t* num_tiles, void* stream) {
    if (!ctx || !sum_tile_lights || !num_tiles) return PBR_ERR_INVALID_ARGUMENT;
    *sum_tile_lights = 0;
    *num_tiles = 0;
    pbr_pass_stats st;
    const int rc = sum_pass_stats(ctx, &st, stream, "pbr_last_cull_stats");
    if (rc != PBR_OK) return rc;
    *sum_tile_lights = st.cull_tile_lights;
    *num_tiles = st.cull_tiles;
    return PBR_OK;
}

int pbr_last_pass_stats(pbr_context* ctx, pbr_pass_stats* out, void* stream) {
    if (!ctx || !out) return PBR_ERR_INVALID_ARGUMENT;
    return sum_pass_stats(ctx, out, stream, "pbr_last_pass_stats");
}

const char* pbr_last_pass_kernel(pbr_context* ctx, void* stream) {
    if (!ctx) return "";
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int si = -1;
    for (size_t i = 0; i < ctx->streams.size(); ++i)
        if (ctx->streams[i].stream == s && ctx->streams[i].tiles > 0) si = (int)i;
    if (si < 0) si = ctx->last_stream;
    return si < 0 ? "" : ctx->streams[si].kernel.c_str();
}

int pbr_debug_bounds(pbr_context* ctx, uint32_t* flags, int reset) {
    if (!ctx) return PBR_ERR_INVALID_ARGUMENT;
    if (!PBR_DEBUG_BOUNDS) return PBR_ERR_UNSUPPORTED;
    DeviceGuard g(ctx->device);
    uint32_t* b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_bounds_mu);
        b = g_bounds_buf[ctx->device];
    }
    if (!g.ok || !b) return PBR_ERR_NOT_READY;
    uint32_t h[2 * pbr::kBoundsClasses];
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h, b, kBoundsBytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) e = hipMemset(b, 0, kBoundsBytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return fail_hip(ctx, e, "pbr_debug_bounds");
    if (flags) std::memcpy(flags, h, kBoundsBytes);
    return PBR_OK;
}

}  // extern "C"

// Development: the balanced pass's per-phase clock sums of a PBR_BAL_PROFILE build (not in the public header).
extern "C" int pbr_debug_bal_profile(unsigned long long* out8, int reset) {
    return pbr::debug_bal_profile(out8, reset != 0) == hipSuccess ? 0 : -1;
}

// Development: per-wave clock stamps of a PBR_WAVE_TIMELINE build into a device buffer of cap_waves * 8 words.
extern "C" int pbr_debug_wave_timeline(void* dev_buf, long long cap_waves) {
    return pbr::debug_wave_timeline(static_cast<unsigned long long*>(dev_buf), cap_waves) == hipSuccess ? 0 : -1;
}
