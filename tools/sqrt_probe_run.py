"""Run tests/hip/sqrt_probe.hip on the GPU: mismatch counts of cheap sqrt sequences vs IEEE sqrtf."""
import ctypes
import os
import subprocess

os.makedirs("build", exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
                "-fhip-fp32-correctly-rounded-divide-sqrt", "-fPIC", "-shared", "-o", "build/sqrt_probe.so",
                "tests/hip/sqrt_probe.hip"], check=True)
L = ctypes.CDLL("build/sqrt_probe.so")
names = ["v_sqrt", "rsq+newton", "v_sqrt+rsq corr", "v_sqrt+rcp corr"]
for w in range(4):
    bad, first = ctypes.c_ulonglong(), ctypes.c_uint()
    rc = L.probe_sqrt(w, -64, 64, ctypes.byref(bad), ctypes.byref(first))
    print(f"{names[w]:18s} exponents [-64,64]: rc {rc} mismatches {bad.value} of {129 << 23} first {first.value:#x}",
          flush=True)
for w, name in enumerate(["1/s by Newton from rsq seed", "1/s by v_rcp + Newton", "1/s by 2 Newton from rsq"]):
    bad, first = ctypes.c_ulonglong(), ctypes.c_uint()
    rc = L.probe_recip_sqrt(w, -64, 64, ctypes.byref(bad), ctypes.byref(first))
    print(f"{name:30s} t exponents [-64,64]: rc {rc} mismatches {bad.value} first {first.value:#x}", flush=True)
