#!/bin/bash
# The CPU test subset under AddressSanitizer + UndefinedBehaviorSanitizer (the reference's debug layer,
# d3dApp.cpp:443-444): `make -C physically_based_renderer_amd/csrc asan` builds the host code with the sanitizers
# (build/asan/), this script runs the tests that drive it -- the G-buffer fill and the C ABI's host half
# (build/asan/libpbrshade.so through PBR_LIB_PATH), the CPU oracle (build/asan/liboracle.so through PBR_ORACLE_LIB)
# -- with clang's shared sanitizer runtime preloaded into Python, then the C example's host half. Any report aborts
# the process (halt_on_error, -fno-sanitize-recover), so a clean run is exit status 0.
# usage: tools/asan_run.sh [extra pytest args]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
make -s -C physically_based_renderer_amd/csrc asan
RT="$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)"
export PBR_LIB_PATH="$ROOT/build/asan/libpbrshade.so" PBR_ORACLE_LIB="$ROOT/build/asan/liboracle.so"
# leaks: CPython and torch keep allocations for the process lifetime by design; the checks that matter here are
# out-of-bounds, use-after-free and undefined behaviour.
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0"
export UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"
LD_PRELOAD="$RT" python -m pytest -q -p no:cacheprovider -m "not gpu" \
  tests/test_host.py tests/test_oracle_golden.py tests/test_known_answers.py tests/test_alpha_test.py \
  tests/test_abi.py "$@"
# The instrumented libraries are the ones loaded, and the sanitizer does report: a G-buffer fill into planes one row
# too short must stop with a heap-buffer-overflow report (a negative control; exit status non-zero expected).
LD_PRELOAD="$RT" python - <<'PY'
import subprocess, sys, textwrap
code = textwrap.dedent("""
    import ctypes
    import numpy as np
    from physically_based_renderer_amd import _native as N, scenes as S
    assert N.LIB_PATH.endswith("build/asan/libpbrshade.so"), N.LIB_PATH
    cfg = S.CONFIGS[2].with_size(64, 8)
    short = [np.zeros(7 * 64, np.float32) for _ in range(N.NUM_PLANES)]  # 7 rows per plane for an 8-row fill
    ptrs = (ctypes.c_void_p * N.NUM_PLANES)(*[p.ctypes.data for p in short])
    d = S._scene_desc(cfg, S.Assets.get())
    N.lib().pbr_gbuffer_fill(ctypes.byref(d), 0, 8, ptrs, 64, 1)
""")
r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
ok = r.returncode != 0 and "heap-buffer-overflow" in r.stderr
print("asan_run: negative control", "detected" if ok else "NOT DETECTED", "-", (r.stderr.strip().splitlines() or [""])[-1][:160])
sys.exit(0 if ok else 1)
PY
build/asan/shade_sphere --host-only --width 97 --height 33
build/asan/shade_sphere --host-only --width 640 --height 360
echo "asan_run: clean"
