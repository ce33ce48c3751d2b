"""The bounds-checked kernel build (PBR_DEBUG_BOUNDS; pbr_debug_bounds.h, `make debug-bounds`) on ragged, strided
frames (tests/bounds_cases.py: 203 x 37 pixels, G-buffer row strides 216 and 221, outputs and coverage planes
with strides of their own) through every kernel family. The reference's debug builds run under the D3D12 debug
layer (d3dApp.cpp:443-444); GPU AddressSanitizer is not available on this pool.

Bars: no index class is ever flagged; every frame is bit-identical to the product library's (a redirected index
would change it); the build's checks do fire -- PBR_DEBUG_BOUNDS_SKEW=1 narrows the output extent the checks use
by one column and must flag class "output" on every pass. The debug library runs in a child process (one library
per process; PBR_LIB_PATH)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bounds_cases

pytestmark = pytest.mark.gpu

ROOT = bounds_cases.ROOT
DEBUG_LIB = bounds_cases.DEBUG_LIB


def _child(tmp_path, name, extra_env=None):
    from physically_based_renderer_amd import _native as N

    if not os.path.exists(DEBUG_LIB):
        pytest.fail(f"{DEBUG_LIB} missing: run `make -C physically_based_renderer_amd/csrc debug-bounds` first")
    # Which library the comparison runs: the bounds-checked build of THIS checkout, or the test stops here (a stale
    # debug build and a real debug/product divergence would otherwise look the same).
    problems = bounds_cases.debug_library_problems(bounds_cases.library_build_info(DEBUG_LIB), N.kernel_sources_sha())
    assert not problems, (f"{DEBUG_LIB} is not the bounds-checked build of this checkout: " + "; ".join(problems)
                          + " (rebuild: make -C physically_based_renderer_amd/csrc debug-bounds)")
    out = tmp_path / f"{name}.npz"
    env = {**os.environ, "PBR_LIB_PATH": DEBUG_LIB, **(extra_env or {})}
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "bounds_cases.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    print(r.stdout.strip())
    z = np.load(out)  # numeric and unicode arrays only: allow_pickle stays False
    return {k.replace("__", "."): z[k] for k in z.files}


def test_product_build_reports_unsupported(gpu):
    from physically_based_renderer_amd import _native as N
    from physically_based_renderer_amd.renderer import ShadingContext

    with ShadingContext(0) as ctx:
        with pytest.raises(N.PbrError) as e:
            ctx.debug_bounds()
        assert e.value.status == N.PBR_ERR_UNSUPPORTED


def test_debug_bounds_clean_and_identical_to_product(tmp_path, gpu):
    dbg = _child(tmp_path, "dbg")
    prod = bounds_cases.run(report_bounds=False)
    frames = [k for k in prod if not k.endswith(".kernel")]
    assert frames and set(frames) <= set(dbg)
    flagged = {k[: -len(".bounds")]: v for k, v in dbg.items() if k.endswith(".bounds") and (v >= 0).any()}
    assert not flagged, f"bounds violations (last index per class gbuffer/output/coverage/texel/light/lds): {flagged}"
    for k in frames:
        assert str(dbg[k + ".kernel"]) == str(prod[k + ".kernel"]), k
        a, b = dbg[k], prod[k]
        assert a.shape == b.shape and a.dtype == b.dtype, k
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), f"{k}: debug build frame differs from product"
    kernels = {str(prod[k + ".kernel"]).split("<")[0] + ("<bal>" if str(prod[k + ".kernel"]).endswith(", 1>") or
                                                           str(prod[k + ".kernel"]).endswith(", 2>") else "")
               for k in frames}
    print(f"{len(frames)} passes, kernel families: {sorted(kernels)}")
    assert {"shade_tile_kernel", "shade_tile_kernel<bal>", "shade_lean_kernel", "shade_tile1_kernel"} <= kernels


def test_debug_bounds_negative_control(tmp_path, gpu):
    dbg = _child(tmp_path, "skew", {"PBR_DEBUG_BOUNDS_SKEW": "1"})
    bounds = {k: v for k, v in dbg.items() if k.endswith(".bounds")}
    assert bounds
    missed = [k for k, v in bounds.items() if v[1] < 0]
    assert not missed, f"output-extent skew not detected in {missed}"
