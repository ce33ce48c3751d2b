"""Which binary a measurement ran (pbr_build_info, ABI 9; VERDICT r04 "what's weak" 4-5).

Every compilation unit of libpbrshade.so carries the stamp of the sources it was compiled from and its build flavor;
bench.py reads them from the library the process LOADED and refuses to publish a number (exit 4, no metric line) for a
development variant, a debug build, a library of other sources or PBR_* development overrides, unless --dev is given.
These tests need no GPU: they link real libraries from the product objects of build/obj with one unit recompiled.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT
import bench
from physically_based_renderer_amd import _native as N

OBJ = os.path.join(ROOT, "build", "obj")
CSRC = os.path.join(ROOT, "physically_based_renderer_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def test_the_in_tree_library_is_the_product_build_of_this_checkout():
    info = N.build_info()
    units = {u["unit"] for u in info["units"]}
    assert units == {"pbr_context", "shade_kernels", "shade_kernels_bal", "gbuffer_fill"}
    assert info["abi"] == N.lib().pbr_abi_version() == 9
    assert info["sources_sha"] == N.kernel_sources_sha() and info["flavor"] == N.PRODUCT_FLAVOR
    assert N.build_problems(info) == []
    sk = next(u for u in info["units"] if u["unit"] == "shade_kernels")
    assert sk["switches"]["PBR_X2_MIN_WAVES"] == "4" and sk["switches"]["PBR_DEBUG_BOUNDS"] == "0"
    assert "max-ilp" in sk["cflags"]  # the unit's own scheduler flag is recorded


def test_build_problems_name_each_kind_of_non_product_build():
    info = N.build_info()
    tree = info["sources_sha"]
    variant = {**info, "flavor": None,
               "units": [dict(u, flavor="variant: x -DPBR_LEAN_MIN_WAVES=5") if u["unit"] == "shade_kernels_bal" else u
                         for u in info["units"]]}
    assert any("variant: x" in p for p in N.build_problems(variant, tree))
    stale = {**info, "units": [dict(u, sources_sha="0" * 16) for u in info["units"]], "sources_sha": "0" * 16}
    assert any("checkout is" in p for p in N.build_problems(stale, tree))
    mixed = {**info, "sources_sha": None,
             "units": [dict(u, sources_sha="0" * 16) if u["unit"] == "gbuffer_fill" else u for u in info["units"]]}
    assert any("different sources" in p for p in N.build_problems(mixed, tree))
    assert N.build_problems({"units": []}, tree)  # a library without build info (ABI < 9)


def _relink(tmp_path, name, defines):
    """The product objects with gbuffer_fill.cpp recompiled under `defines` (the fastest unit to rebuild)."""
    if not all(os.path.exists(os.path.join(OBJ, f)) for f in ("shade_kernels.o", "shade_kernels_bal.o", "pbr_context.o")):
        pytest.skip("product objects not built (build/obj)")
    obj = tmp_path / f"{name}_gbuffer_fill.o"
    so = tmp_path / name / "libpbrshade.so"
    so.parent.mkdir()
    subprocess.run([HIPCC, "-O1", "-std=c++17", "-fPIC", f"-I{ROOT}/include", f"-I{CSRC}", *defines, "-x", "c++", "-c",
                    os.path.join(CSRC, "gbuffer_fill.cpp"), "-o", str(obj)], check=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-o", str(so), os.path.join(OBJ, "shade_kernels.o"),
                    os.path.join(OBJ, "shade_kernels_bal.o"), os.path.join(OBJ, "pbr_context.o"), str(obj),
                    "-lpthread"], check=True)
    return str(so)


def _bench(lib, *extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("PBR_")}
    env["PBR_LIB_PATH"] = lib
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", *extra],
                          capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)


@pytest.mark.parametrize("kind", ["variant", "stale"])
def test_bench_refuses_a_variant_or_stale_library(kind, tmp_path):
    """bench.py exits 4 with no metric line when the library it loads is a development variant (a unit stamped
    "variant: ... -DPBR_BAL_EXPERIMENT=4", as tools/build_variant.sh stamps them) or was built from other sources
    than the checkout (a stale .so); the refusal names the reason. (With --dev it would go on to measure: on this
    GPU-less host it then stops at the missing device, exit 1, after the provenance check.)"""
    sha = N.kernel_sources_sha()
    if kind == "variant":
        defines = [f'-DPBR_SOURCES_SHA="{sha}"', '-DPBR_BUILD_FLAVOR="variant: x -DPBR_BAL_EXPERIMENT=4"', "-DPBR_BAL_EXPERIMENT=4"]
        reason = "variant: x -DPBR_BAL_EXPERIMENT=4"
    else:
        defines = ['-DPBR_SOURCES_SHA="0123456789abcdef"', '-DPBR_BUILD_FLAVOR="product"']
        reason = "different sources"
    lib = _relink(tmp_path, kind, defines)
    r = _bench(lib)
    assert r.returncode == bench.EXIT_PROVENANCE, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "REFUSED" in r.stderr and reason in r.stderr
    r = _bench(lib, "--dev")
    assert r.returncode != bench.EXIT_PROVENANCE and "REFUSED" not in r.stderr


def test_debug_bounds_comparison_refuses_a_restamped_or_product_library(tmp_path):
    """tests/test_gpu_debug_bounds.py compares frames only after checking WHICH library its child loads: every unit
    stamped with this checkout's sources and the kernel units built as debug_bounds. A library with one unit restamped
    (a stale `make debug-bounds`) and the product library are both refused, with the reason named; the in-tree debug
    library passes when it is present and current."""
    import bounds_cases as B

    tree = N.kernel_sources_sha()
    stale = _relink(tmp_path, "stale_dbg", ['-DPBR_SOURCES_SHA="0123456789abcdef"', '-DPBR_BUILD_FLAVOR="product"'])
    p = B.debug_library_problems(B.library_build_info(stale), tree)
    assert any("unit gbuffer_fill built from sources 0123456789abcdef" in s for s in p), p
    assert any("is a 'product' build, not 'debug_bounds'" in s for s in p), p
    p = B.debug_library_problems(B.library_build_info(N.LIB_PATH), tree)
    assert p and all("'product' build" in s for s in p), p
    assert B.debug_library_problems({"units": []}, tree)
    # a debug library whose kernel units carry an older stamp (the round-5 failure's cause)
    info = {"units": [{"unit": u, "sources_sha": "ffffffffffffffff", "flavor": B.DEBUG_FLAVOR} for u in B.DEBUG_UNITS]
            + [{"unit": "gbuffer_fill", "sources_sha": tree, "flavor": "product"}]}
    p = B.debug_library_problems(info, tree)
    assert len(p) == 3 and all("ffffffffffffffff" in s for s in p)
    if os.path.exists(B.DEBUG_LIB):
        info = B.library_build_info(B.DEBUG_LIB)
        if info["sources_sha"] == tree or all(u["sources_sha"] == tree for u in info["units"]):
            assert B.debug_library_problems(info, tree) == []


def test_bench_records_the_loaded_library():
    """library_provenance describes the loaded build in the line (path, stamp, flavor, units) and lists problems."""
    lib = bench.library_provenance(False)
    assert lib["path"] == os.path.join("physically_based_renderer_amd", "_lib", "libpbrshade.so")
    assert lib["sources_sha"] == lib["tree_sources_sha"] == N.kernel_sources_sha()
    assert lib["flavor"] == "product" and len(lib["units"]) == 4
    overrides = [k for k in os.environ if k.startswith("PBR_") and k not in bench.ENV_NEUTRAL]
    assert bool(lib["problems"]) == bool(overrides)
