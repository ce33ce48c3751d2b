"""Run tests/hip/seed_div_probe.hip on the GPU (development probe): is the Markstein quotient a / s
still RN(a / s) when the reciprocal comes from the rsq seed of s = RN(sqrt(t)) instead of v_rcp?

    python tools/seed_div_probe_run.py            # t exponents [-64, 64]
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "build", "seed_div_probe.so")
os.makedirs(os.path.dirname(SO), exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
                "-fhip-fp32-correctly-rounded-divide-sqrt", "-fPIC", "-shared", "-o", SO,
                os.path.join(ROOT, "tests", "hip", "seed_div_probe.hip")], check=True)
if "--build-only" in sys.argv:
    sys.exit(0)
L = ctypes.CDLL(SO)
cap = 4096
out = (ctypes.c_ulonglong * 6)()
lst = (ctypes.c_uint32 * cap)()
first = ctypes.c_uint32()
rc = L.probe_seed_div(-64, 64, out, lst, cap, ctypes.byref(first))
n = min(out[3], cap)
print(f"rc {rc}; t exponents [-64, 64] ({129 << 23} values): sqrt_nr != sqrtf {out[0]}, recip_nr != 1/s {out[1]}, "
      f"seeded reciprocal != 1/s {out[2]}")
sig = sorted({(ctypes.c_float.from_buffer_copy(ctypes.c_uint32(lst[i])).value) for i in range(min(n, 8))})
print("first listed t:", [f"{v:.9g}" for v in sig])
print(f"quotients a / s over the listed t: {out[5]} tested (x2 signs), {out[4]} Markstein mismatches"
      + (f", first failing t bits {first.value:#x}" if out[4] else ""))
