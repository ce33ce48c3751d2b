// pbr_debug_bounds.h -- the bounds-checked kernel build (PBR_DEBUG_BOUNDS=1; `make debug-bounds` builds it into
// _lib/debug_bounds/libpbrshade.so). The D3D12 debug layer the reference enables in debug builds
// (d3dApp.cpp:443-444) validates resource accesses; GPU AddressSanitizer is not available on this pool, so this
// build checks every global index the shading kernels form -- G-buffer pixel reads (pixel inside the frame, row
// stride respected), output and coverage offsets, sky / environment texel indices, light records
// -- and the balanced lists' LDS indices, against the extents the launch was given.
//
// A violation does not trap (a faulting or trapped wave can take every GPU of the host down): it sets the class's
// word in a device flag buffer with a plain vector store, records the offending index (last writer wins) and
// replaces the index by 0, so the kernel finishes and the host reads the flags (pbr_debug_bounds). Product builds
// (PBR_DEBUG_BOUNDS unset) compile every check to the index itself: their code objects are unchanged.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef PBR_DEBUG_BOUNDS
#define PBR_DEBUG_BOUNDS 0
#endif

namespace pbr {

// Index classes (words of the flag buffer; word kBoundsClasses + c: the last offending index of class c).
enum BoundsClass {
    kBoundsGBuffer = 0,   // G-buffer plane read: pixel (x, y) inside width x height, index y * row_stride + x
    kBoundsOutput = 1,    // output store: same pixel rule with out_stride
    kBoundsCoverage = 2,  // coverage byte read
    kBoundsTexel = 3,     // sky / environment texel (y * w + x < w * h)
    kBoundsLight = 4,     // light record (j < n_dir + n_point + n_spot)
    kBoundsLds = 5,       // balanced lists: light index <= kBalMaxLights (the zero sentinel), list slot < 128
    kBoundsClasses = 8
};

#if PBR_DEBUG_BOUNDS
// One per translation unit (each kernel TU publishes its own copy; debug_bounds() points both at one buffer).
static __device__ uint32_t* g_bounds_flags;

[[maybe_unused]] static __device__ __noinline__ void bounds_violation(int64_t i, int cls) {
    uint32_t* f = g_bounds_flags;
    if (f != nullptr) {
        f[cls] = 1u;
        f[kBoundsClasses + cls] = (uint32_t)i;
    }
}
// i in [0, n); otherwise flagged and 0.
__device__ __forceinline__ int64_t bounds_linear(int64_t i, int64_t n, int cls) {
    if (__builtin_expect(i < 0 || i >= n, 0)) {
        bounds_violation(i, cls);
        return 0;
    }
    return i;
}
// i = y * stride + x with 0 <= y < h and 0 <= x < w (span elements from i, for paired loads); otherwise flagged
// and 0.
__device__ __forceinline__ int64_t bounds_pixel(int64_t i, int w, int h, int64_t stride, int span, int cls) {
    const int64_t y = stride > 0 ? i / stride : 0, x = i - y * stride;
    if (__builtin_expect(i < 0 || y >= h || x + span > w, 0)) {
        bounds_violation(i, cls);
        return 0;
    }
    return i;
}
#define PBR_BOUNDS(i, n, cls) ::pbr::bounds_linear((i), (n), (cls))
#define PBR_BOUNDS_PIXEL(i, w, h, stride, span, cls) ::pbr::bounds_pixel((i), (w), (h), (stride), (span), (cls))
#else
#define PBR_BOUNDS(i, n, cls) (i)
#define PBR_BOUNDS_PIXEL(i, w, h, stride, span, cls) (i)
#endif

}  // namespace pbr
