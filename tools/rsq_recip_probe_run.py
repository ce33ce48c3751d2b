"""Run tests/hip/rsq_recip_probe.hip on the GPU: which three-operation reciprocals of s = RN(sqrt(t)) from the square
root's own v_rsq seed equal RN(1 / s) for every t with exponent in [emin, emax] (development tool).
usage: python tools/rsq_recip_probe_run.py [emin emax]"""
import ctypes
import os
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
so = os.path.join(ROOT, "build", "rsq_recip_probe.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
                "-fhip-fp32-correctly-rounded-divide-sqrt", "-fPIC", "-shared", "-o", so,
                os.path.join(ROOT, "tests", "hip", "rsq_recip_probe.hip")], check=True)
L = ctypes.CDLL(so)
emin, emax = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (-64, 64)
names = ["v_rcp + Newton (control)", "1 Newton from rsq", "2 Newton from rsq", "Newton + e^2 term", "Newton, refined product", "Newton, seed one ulp up", "Newton, e (1 + 2^-23)"]
f = lambda u: struct.unpack("<f", struct.pack("<I", u))[0]  # noqa: E731
for w, name in enumerate(names):
    bad = ctypes.c_ulonglong()
    log = (ctypes.c_uint32 * 64)()
    rc = L.probe_rsq_recip(w, emin, emax, ctypes.byref(bad), log, 16)
    print(f"{w} {name:26s} t exponents [{emin},{emax}]: rc {rc} mismatches {bad.value} of {(emax - emin + 1) << 23}",
          flush=True)
    for k in range(min(bad.value, 4)):
        t, s, r, want = log[4 * k: 4 * k + 4]
        print(f"    t {f(t)!r} ({t:#010x}) s {f(s)!r} ({s:#010x}) r {r:#010x} want {want:#010x}", flush=True)
