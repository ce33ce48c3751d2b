"""Ragged, strided frames through every kernel family, for tests/test_gpu_debug_bounds.py.

Run in-process against the product library, and as a child process (`python tests/bounds_cases.py OUT.npz`)
against the bounds-checked build (PBR_LIB_PATH=physically_based_renderer_amd/_lib/debug_bounds/libpbrshade.so), which then also stores the
pbr_debug_bounds report of every case. The frames are 203 x 37 pixels (odd width: the last pixel pair has one
pixel; 37 rows: the last tile is partial) in G-buffers whose row stride is 216 (even: the 8-byte pair loads) or
221 (odd: the per-pixel loads), written into outputs and read from coverage planes with strides of their own.
The cases cover the kernel families -- the pair kernel (uniform, culled, wave-balanced faithful and exact
lists), the lean pair kernel, the one-pixel kernel (PBR_PIXELS_PER_THREAD=1), the non-lean pair kernel
(PBR_LEAN=0) -- with constant and IBL ambient, F0 plane, AO, EXACT_ONLY, the sky pass (RGBA32F and RGBA8) and
the ALPHA_TEST permutation.
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

W, H = 203, 37
STRIDES = (216, 221)
# Context settings (read by pbr_context_create): the default layout, the one-pixel kernel, no lean kernel.
LAYOUTS = {"pair": {}, "px1": {"PBR_PIXELS_PER_THREAD": "1"}, "nolean": {"PBR_LEAN": "0"}}


DEBUG_LIB = os.path.join(ROOT, "physically_based_renderer_amd", "_lib", "debug_bounds", "libpbrshade.so")
DEBUG_FLAVOR = "debug_bounds"
# The units `make debug-bounds` compiles with -DPBR_DEBUG_BOUNDS=1; the G-buffer fill is the product object (host code).
DEBUG_UNITS = ("shade_kernels", "shade_kernels_bal", "pbr_context")


def library_build_info(lib_path: str) -> dict:
    """pbr_build_info of the library at `lib_path`, read in a child process (one libpbrshade.so per process; loading it
    touches no GPU)."""
    import json
    import subprocess

    code = ("import json, sys; sys.path.insert(0, %r); from physically_based_renderer_amd import _native as N; "
            "print(json.dumps(N.build_info()))" % ROOT)
    env = {**os.environ, "PBR_LIB_PATH": lib_path}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        raise RuntimeError(f"cannot read the build info of {lib_path}: {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def debug_library_problems(info: dict, tree_sha: str) -> list:
    """Why a library is not the bounds-checked build of this checkout (empty = it is): a unit stamped with other
    sources than the checkout's (a stale `make debug-bounds`: round 5's pass-2 log compared such a library with the
    product), or a kernel unit that is not a debug_bounds build (the product library, a variant)."""
    bad = []
    if not info.get("units"):
        return ["the library reports no build info (ABI < 9)"]
    for u in info["units"]:
        if u["sources_sha"] != tree_sha:
            bad.append(f"unit {u['unit']} built from sources {u['sources_sha']}, checkout is {tree_sha}")
        if u["unit"] in DEBUG_UNITS and u["flavor"] != DEBUG_FLAVOR:
            bad.append(f"unit {u['unit']} is a {u['flavor']!r} build, not {DEBUG_FLAVOR!r}")
    missing = set(DEBUG_UNITS) - {u["unit"] for u in info["units"]}
    if missing:
        bad.append(f"units missing: {sorted(missing)}")
    return bad


def _cases():
    from physically_based_renderer_amd import _native as N

    F, AO, X, CULL = N.PBR_FLAG_FAITHFUL, N.PBR_FLAG_APPLY_AO, N.PBR_FLAG_EXACT_ONLY, N.PBR_FLAG_TILED_CULLING
    # (name, config id, flags added, flags removed, frame path with sky, RGBA8, alpha test)
    return [
        ("cfg1_frame_sky", 1, 0, 0, True, False, False),
        ("cfg1_frame_sky_rgba8", 1, F, 0, True, True, False),
        ("cfg2", 2, 0, 0, False, False, False),
        ("cfg2_faithful_ao", 2, F | AO, 0, False, False, False),
        ("cfg2_culled", 2, CULL, 0, False, False, False),
        ("cfg3_faithful", 3, F, 0, False, False, False),        # wave-balanced faithful lists + packed IBL
        ("cfg3_exact", 3, 0, 0, False, False, False),
        ("cfg3_exact_only", 3, X, 0, False, False, False),
        ("cfg3_faithful_alpha", 3, F, 0, False, False, True),
        ("cfg4_faithful", 4, F, 0, False, False, False),        # 256 lights, tiled culling, F0 plane
        ("cfg4_uniform_ao", 4, AO, CULL, False, False, False),
        ("cfg4_frame_rgba8", 4, 0, 0, True, True, False),
    ]


def _balanced_exact_pass(pc):
    """cfg3's exact pass without directional lights: the wave-balanced EXACT lists (PassArgs::balanced 2)."""
    from physically_based_renderer_amd.renderer import PassConstants

    d = {**pc.__dict__}
    nd = int(d["num_dir_lights"])
    d["lights_array"] = np.ascontiguousarray(pc.light_array()[nd:])
    d["num_dir_lights"] = 0
    return PassConstants(**d)


def run(report_bounds: bool):
    """{case: output array, case + '.kernel': the kernel it launched} and, with report_bounds, {case + '.bounds':
    int64[6]} -- the last offending index per class, -1 where the class was clean."""
    import torch

    from physically_based_renderer_amd import _native as N
    from physically_based_renderer_amd import envmap
    from physically_based_renderer_amd import scenes as S
    from physically_based_renderer_amd.renderer import GBuffer, PassConstants, ShadingContext

    dev = torch.device("cuda", 0)
    sky = envmap.procedural_sky_rgba16()
    env = S.env_map()
    classes = ("gbuffer", "output", "coverage", "texel", "light", "lds")
    results = {}
    for layout, env_vars in LAYOUTS.items():
        saved = {k: os.environ.get(k) for k in env_vars}
        os.environ.update(env_vars)
        try:
            ctx = ShadingContext(0)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        if report_bounds:
            ctx.debug_bounds(reset=True)
        for name, cid, add, remove, frame, rgba8, alpha in _cases():
            cfg = S.CONFIGS[cid].with_size(W, H)
            planes, cov = S.fill_gbuffer_host_coverage(cfg)
            pc = S.scene_pass(cfg)
            pc = PassConstants(**{**pc.__dict__, "flags": (pc.flags | add | (N.PBR_FLAG_ALPHA_TEST if alpha else 0))
                                  & ~remove})
            if name == "cfg3_exact":
                pc = _balanced_exact_pass(pc)
            for stride in STRIDES:
                t = torch.zeros((N.NUM_PLANES, H, stride), dtype=torch.float32)
                t[:, :, :W] = torch.from_numpy(planes)
                opacity = None
                if alpha:
                    rng = np.random.default_rng(cid * 1000 + stride)
                    o = torch.zeros((H, stride), dtype=torch.float32)
                    o[:, :W] = torch.from_numpy(rng.uniform(-0.2, 1.0, (H, W)).astype(np.float32))
                    opacity = o.to(dev)
                gb = GBuffer(t.to(dev), width=W, opacity=opacity)
                ctx.set_pass(pc)
                if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE:
                    ctx.set_env_map(env)
                key = f"{layout}.{name}.s{stride}"
                if frame:
                    ctx.set_sky_map(sky)
                    c = torch.zeros((H, W + 7), dtype=torch.uint8)
                    c[:, :W] = torch.from_numpy(cov)
                    dt = torch.uint8 if rgba8 else torch.float32
                    out = torch.full((H, W + 5, 4), 7, dtype=dt, device=dev)[:, :W]
                    ctx.shade_frame(gb, out=out, coverage=c.to(dev)[:, :W],
                                    fmt=N.PBR_OUTPUT_RGBA8_UNORM if rgba8 else N.PBR_OUTPUT_RGBA32F)
                else:
                    out = torch.full((H, W + 5, 4), 7.0, dtype=torch.float32, device=dev)[:, :W]
                    ctx.shade(gb, out=out)
                torch.cuda.synchronize()
                results[key] = np.ascontiguousarray(out.cpu().numpy())
                results[key + ".kernel"] = np.array(ctx.last_kernel())
                if report_bounds:
                    bad = ctx.debug_bounds(reset=True)
                    results[key + ".bounds"] = np.array([bad.get(n, -1) for n in classes], np.int64)
        ctx.close()
    return results


if __name__ == "__main__":
    out_path = sys.argv[1]
    res = run(report_bounds=True)
    np.savez(out_path, **{k.replace(".", "__"): v for k, v in res.items()})
    print(f"bounds_cases: {sum(1 for k in res if k.endswith('.bounds'))} passes", flush=True)
