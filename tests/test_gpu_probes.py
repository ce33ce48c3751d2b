"""Device-level proofs behind the kernel's exactness claims ("exact fast path"):

* fastdiv_probe.hip -- v_rcp_f32 + one Newton step is RN(1/b) for every b with exponent in
  [-64, 64] (the window the fast path admits), and the Markstein quotient equals IEEE a / b on
  random operands inside the window;
* quarter_dot_probe.hip -- the faithful loop's power-of-two rescaled invariants (faithful_scale): N/4 . H
  is exactly N.H / 4 in the fast window, so the dot's clamp bit gives max(N.H, 0) / 4 in lean waves, the
  GGX denominator keeps the reference's bits, and faithful_unscale restores every invariant;
* wave_ops_probe.hip -- the DPP wave reductions and scan of pbr_device_math_x2.h (the culling box, pass 1's box and
  bounds, the balanced ranking's prefix sum) against a serial evaluation;
* libm_probe.hip -- the device build of libm_f32.h (WorldToSkyUV's atan2f / asinf) returns the host
  glibc's bits: asinf on every float in [-1, 1], atanf on every finite float, and 2^27 random
  atan2f pairs.

Both are compiled here with the product's fp flags (csrc/Makefile FPFLAGS).
"""
import ctypes
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "-std=c++17", "-Wno-unused-value", "-Wno-unused-result", "-fPIC", "-shared", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-I", os.path.join(ROOT, "physically_based_renderer_amd", "csrc")]


@pytest.fixture(scope="module")
def probes(tmp_path_factory, gpu):
    d = tmp_path_factory.mktemp("probes")
    libs = {}
    for name in ("fastdiv_probe", "libm_probe", "sqrt_probe", "gamma_probe", "quarter_dot_probe", "wave_ops_probe"):
        so = str(d / f"{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, os.path.join(ROOT, "tests", "hip", f"{name}.hip"), "-o", so,
                        "-lpthread"], check=True)
        libs[name] = ctypes.CDLL(so)
    return libs


def test_reciprocal_is_correctly_rounded_in_window(probes):
    L = probes["fastdiv_probe"]
    bad, first = ctypes.c_ulonglong(), ctypes.c_uint()
    assert L.probe_recip(-64, 64, ctypes.byref(bad), ctypes.byref(first)) == 0
    assert bad.value == 0, hex(first.value)


def test_rsq_newton_sqrt_is_ieee_in_window(probes):
    """The fast path's sqrt (v_rsq + one Newton step, pbr_device_math.h sqrt_nr) equals IEEE sqrtf for
    every float with exponent in [-64, 64]; bare v_sqrt_f32 does not (kept as a control)."""
    L = probes["sqrt_probe"]
    bad, first = ctypes.c_ulonglong(), ctypes.c_uint()
    assert L.probe_sqrt(1, -64, 64, ctypes.byref(bad), ctypes.byref(first)) == 0
    assert bad.value == 0, hex(first.value)
    assert L.probe_sqrt(0, -64, 64, ctypes.byref(bad), ctypes.byref(first)) == 0
    assert bad.value > 0


def test_div_pi_is_ieee_on_device(probes):
    """The fast path's 2-op division by PI over the window's magnitudes [2^-98, 2^100], both signs."""
    L = probes["fastdiv_probe"]
    bad = ctypes.c_ulonglong()
    assert L.probe_div_pi(-98, 100, ctypes.byref(bad)) == 0
    assert bad.value == 0


@pytest.mark.parametrize("alo,ahi,blo,bhi", [(-96, 60, -60, 60), (-30, 30, -30, 30), (-5, 5, -5, 5)])
def test_markstein_quotient_is_ieee(probes, alo, ahi, blo, bhi):
    L = probes["fastdiv_probe"]
    bad, bad_r, ex = ctypes.c_ulonglong(), ctypes.c_ulonglong(), (ctypes.c_float * 2)()
    assert L.probe_div(ctypes.c_ulonglong(777 + alo), 65536, 16, alo, ahi, blo, bhi, ctypes.byref(bad),
                       ctypes.byref(bad_r), ex) == 0
    assert bad.value == 0 and bad_r.value == 0, (ex[0], ex[1])


@pytest.mark.parametrize("which,ranges", [(0, [(0, 0x3F800000), (0x80000000, 0xBF800000)]),
                                          (1, [(0, 0x7F7FFFFF), (0x80000000, 0xFF7FFFFF)])])
def test_device_libm_port_equals_glibc(probes, which, ranges):
    L = probes["libm_probe"]
    L.probe_unary.restype = ctypes.c_longlong
    L.probe_unary.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    for lo, hi in ranges:
        first = ctypes.c_uint32()
        bad = L.probe_unary(which, lo, hi, ctypes.byref(first))
        assert bad == 0, f"{['asinf', 'atan2f(y,1)'][which]}: {bad} mismatches, first 0x{first.value:08x}"


def test_device_atan2f_pairs_equal_glibc(probes):
    L = probes["libm_probe"]
    L.probe_atan2_pairs.restype = ctypes.c_longlong
    L.probe_atan2_pairs.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float),
                                    ctypes.POINTER(ctypes.c_float)]
    y, x = ctypes.c_float(), ctypes.c_float()
    bad = L.probe_atan2_pairs(2024, 1 << 27, ctypes.byref(y), ctypes.byref(x))
    assert bad == 0, f"{bad} mismatches, first atan2f({y.value!r}, {x.value!r})"


@pytest.mark.parametrize("which,ranges", [(0, [(0, 0x3F800000 + 0x100000), (0x80000000, 0xBF800000 + 0x100000)]),
                                          (1, [(0, 0x7F7FFFFF), (0x80000000, 0xFF7FFFFF)])])
def test_device_libm_pair_forms_equal_glibc(probes, which, ranges):
    """The branch-free pair forms (libm_f32_x2.h: pbr_asinf_x2 over every float in [-1, 1] and a stretch past it,
    pbr_atan2f_x2(y, 1) over every finite y), evaluated on the device two arguments per work-item: glibc's bits
    wherever they do not flag an element special, and flagged exactly where the scalar function is needed
    (|x| > 1 / NaN; atan2f components outside 0 or [2^-40, 2^40])."""
    L = probes["libm_probe"]
    L.probe_unary_x2.restype = ctypes.c_longlong
    L.probe_unary_x2.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    for lo, hi in ranges:
        first = ctypes.c_uint32()
        bad = L.probe_unary_x2(which, lo, hi, ctypes.byref(first))
        assert bad == 0, f"{['asinf_x2', 'atan2f_x2(y,1)'][which]}: {bad} mismatches, first 0x{first.value:08x}"


def test_device_atan2f_pair_form_random_pairs_equal_glibc(probes):
    L = probes["libm_probe"]
    L.probe_atan2_pairs_x2.restype = ctypes.c_longlong
    L.probe_atan2_pairs_x2.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float),
                                       ctypes.POINTER(ctypes.c_float)]
    y, x = ctypes.c_float(), ctypes.c_float()
    bad = L.probe_atan2_pairs_x2(2025, 1 << 27, ctypes.byref(y), ctypes.byref(x))
    assert bad == 0, f"{bad} mismatches, first atan2f({y.value!r}, {x.value!r})"


def test_faithful_gamma_error_exhaustive(probes):
    """PBR_FLAG_FAITHFUL's gamma encode vs the host glibc powf(c, 1/2.2f) on every float of the binades
    [2^-40, 1): within 5.4e-7 relative (9 x 2^-24) from 2^-10 up and 1.05e-6 down to 2^-32, where the hardware
    exp2/log2 path runs; bit-identical below it (the glibc algorithm). DESIGN.md §2 adds this to the faithful
    bound. (c = 0 takes the hardware path too: +0, as powf; the full-frame parity tests cover it.)"""
    L = probes["gamma_probe"]
    lo, hi = -40, -1
    out = (ctypes.c_double * (hi - lo + 1))()
    assert L.probe_gamma(lo, hi, out) == 0
    for e in range(lo, hi + 1):
        print(f"binade 2^{e}: max_rel {out[e - lo]:.3g}")
        if e >= -10:
            assert out[e - lo] <= 5.4e-7, e
        elif e >= -32:
            assert out[e - lo] <= 1.05e-6, e
        else:
            assert out[e - lo] == 0.0, e


@pytest.mark.parametrize("lean", [1, 0])
def test_faithful_quarter_dots_are_exact(probes, lean):
    """faithful_scale's claim (pbr_device_math_x2.h): over 2^24 random pixel pairs in the fast window --
    H near N (N.H ~ 1, where the GGX denominator cancels), components forced to 0 or to the window's small
    ends -- the rescaled dot is the reference's dot / 4 bit for bit (clamp bit in lean waves, max
    elsewhere), the GGX denominator from it has the reference's bits, and unscaling is exact."""
    L = probes["quarter_dot_probe"]
    bad = (ctypes.c_ulonglong * 4)()
    assert L.probe_quarter_dots(ctypes.c_ulonglong(0x9A4D + lean), 4096, 16, lean, bad) == 0
    assert list(bad[:3]) == [0, 0, 0]
    if lean:  # control: the samples reach N.H > 1, where saturating the unscaled dot would have clamped
        assert bad[3] > 0


def test_dpp_wave_reductions_and_scan(probes):
    """wave_min_dpp / wave_max_dpp (integer keys, NaN counted as the neutral value, as fminf / fmaxf ignore it),
    wave_sum_dpp and the inclusive wave_scan_add_dpp against numpy, on waves of random floats over many binades with
    +-0, +-inf, NaN and denormals mixed in, one wave all NaN (-> the neutral values), and random ints."""
    import numpy as np

    rng = np.random.default_rng(2024)
    n = 4096
    f = (rng.standard_normal(64 * n) * np.exp2(rng.integers(-60, 60, 64 * n))).astype(np.float32)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3.0e38, -3.0e38], np.float32)
    pick = rng.random(64 * n) < 0.05
    f[pick] = rng.choice(specials, pick.sum())
    f[64 * 7:64 * 8] = np.nan
    iv = rng.integers(-1000, 1000, 64 * n).astype(np.int32)
    mn, mx = np.empty(n, np.float32), np.empty(n, np.float32)
    sm, sc = np.empty(n, np.int32), np.empty(64 * n, np.int32)
    P = ctypes.POINTER
    fn = probes["wave_ops_probe"].probe_wave_ops
    assert fn(f.ctypes.data_as(P(ctypes.c_float)), iv.ctypes.data_as(P(ctypes.c_int)), n,
              mn.ctypes.data_as(P(ctypes.c_float)), mx.ctypes.data_as(P(ctypes.c_float)),
              sm.ctypes.data_as(P(ctypes.c_int)), sc.ctypes.data_as(P(ctypes.c_int))) == 0
    w = f.reshape(n, 64)
    want_mn = np.where(np.isnan(w), np.float32(3.0e38), w).min(axis=1)
    want_mx = np.where(np.isnan(w), np.float32(-3.0e38), w).max(axis=1)
    assert np.array_equal(mn, want_mn) and np.array_equal(mx, want_mx)  # -0 == +0 here; the values are the point
    assert mn[7] == np.float32(3.0e38) and mx[7] == np.float32(-3.0e38)
    assert np.array_equal(sm, iv.reshape(n, 64).sum(axis=1))
    assert np.array_equal(sc, np.cumsum(iv.reshape(n, 64), axis=1).reshape(-1))
