"""Host-side checks of the profiling tools whose output the bench line quotes (tools/pmc_summarize.py)."""
import csv
import importlib.util
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def load_tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_counters_average_the_workloads_own_dispatches(tmp_path):
    """bench.py at N = 1 also shades the scaling anchor (another kernel, another grid) after the timed steps:
    the summary must average the workload's first six shading dispatches only, whichever pair kernel ran."""
    pmc = load_tool("pmc_summarize")
    path = tmp_path / "pmc_counter_collection.csv"
    fields = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        w.writerow({"Dispatch_Id": 1, "Kernel_Name": "__amd_rocclr_copyBuffer", "Counter_Name": "FETCH_SIZE",
                    "Counter_Value": 1e9})
        for d in range(2, 8):  # the workload: lean kernel, 100 KiB per launch
            w.writerow({"Dispatch_Id": d, "Kernel_Name": "void pbr::shade_lean_kernel<0, false, false, false, true>(...)",
                        "Counter_Name": "FETCH_SIZE", "Counter_Value": 100.0})
        for d in range(8, 16):  # the scale anchor: a balanced kernel, 190 KiB per launch
            w.writerow({"Dispatch_Id": d, "Kernel_Name": "void pbr::shade_tile_kernel<1, false, false, false, 1>(...)",
                        "Counter_Name": "FETCH_SIZE", "Counter_Value": 190.0})
    assert pmc.per_kernel(str(path)) == {"FETCH_SIZE": 100.0}


def test_profile_stamp_comes_from_the_loaded_library():
    """A profile is stamped with the library the profiled bench process loaded (its line's `library`, pbr_build_info),
    and a development / debug / stale build is refused rather than stamped."""
    import pytest

    pmc = load_tool("pmc_summarize")
    lib = {"path": "physically_based_renderer_amd/_lib/libpbrshade.so", "sources_sha": "abcd" * 4, "flavor": "product",
           "tree_sources_sha": "abcd" * 4, "problems": []}
    sha, rec = pmc.library_stamp({"library": lib})
    assert sha == "abcd" * 4 and rec["flavor"] == "product"
    for bad in ({"library": {**lib, "problems": ["unit shade_kernels_bal is a 'variant: x' build"]}},
                {"library": {**lib, "sources_sha": None}}, {}, None):
        with pytest.raises(SystemExit):
            pmc.library_stamp(bad)


def test_phase_census_splits_phases_weights_loops_and_skips_cold_paths(tmp_path, capsys):
    """tools/isa_census_phases.py on a hand-written kernel: two phases, a divergent `if` (counted), a uniform fallback
    that starts with a cold marker (not counted), an IEEE-division block (cold by content, not counted) and a loop
    weighted by its iteration count per wave."""
    census = load_tool("isa_census_phases")
    asm = """_Zk:
; %bb.0:
\t;;#ASMSTART
\t; @phase entry
\t;;#ASMEND
\tv_add_u32_e32 v1, v2, v3
\tv_cmp_gt_u32_e32 vcc, 5, v0
\ts_and_saveexec_b64 s[4:5], vcc
\ts_cbranch_execz .LBB0_2
; %bb.1:
\tv_pk_mul_f32 v[2:3], v[2:3], v[4:5]
.LBB0_2:
\ts_or_b64 exec, exec, s[4:5]
\ts_cmp_eq_u32 s6, 0
\ts_cbranch_scc1 .LBB0_4
; %bb.3:
\t;;#ASMSTART
\t; @phase cold_fallback
\t;;#ASMEND
\tv_div_scale_f32 v1, s[6:7], v2, v2, v3
\ts_branch .LBB0_5
.LBB0_4:
\tv_mov_b32_e32 v9, 0
.LBB0_5:
\t;;#ASMSTART
\t; @phase loop
\t;;#ASMEND
\tv_mov_b32_e32 v8, 0
.LBB0_6:                                ; =>This Inner Loop Header: Depth=1
\tv_pk_fma_f32 v[2:3], v[2:3], v[4:5], v[6:7]
\tv_rcp_f32_e32 v1, v2
\ts_cbranch_scc1 .LBB0_6
; %bb.7:
\t;;#ASMSTART
\t; @phase tail
\t;;#ASMEND
\tv_add_f32_e32 v1, v2, v3
\ts_endpgm
.Lfunc_end0:
"""
    path = tmp_path / "k.s"
    path.write_text(asm)
    import sys

    argv = sys.argv
    sys.argv = ["isa_census_phases.py", str(path), "--kernel", "_Zk", "--path", "entry", "loop", "tail",
                "--weights", "loop=10"]
    try:
        census.main()
    finally:
        sys.argv = argv
    out = capsys.readouterr().out
    rows = {l.split()[0]: l.split() for l in out.splitlines() if l.split() and l.split()[0] in ("entry", "loop", "tail")}
    # entry: v_add, v_cmp, the divergent v_pk_mul and the fall-through v_mov (the uniform branch's two sides: the cold
    # side stops at its marker) -> the always + divergent count; the cold v_div_scale is not counted
    assert int(rows["entry"][-5]) == 4, out
    # loop: 2 VALU per iteration x 10 + the v_mov before the loop once
    assert float(rows["loop"][-2]) == 2 * 10, out
    assert int(rows["tail"][-5]) == 1, out
    total = [l for l in out.splitlines() if l.startswith("total")][0].split()
    assert float(total[1]) == 4 + 20 + 1 + 1
