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
