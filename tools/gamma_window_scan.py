"""Development: the faithful gamma encode's error per binade with the hardware path extended down to 2^-60
(PBR_FAITHFUL_GAMMA_LO), to choose the window (profiles/r04/gamma_window_scan.log). Runs on the GPU box; prints one line per binade."""
import ctypes, subprocess, os, sys
ROOT="/root/repo" if os.path.exists("/root/repo") else os.getcwd()
so=os.path.join(os.environ.get("TMPDIR", "/tmp"), "gamma_probe_lo.so")
subprocess.run(["/opt/rocm/bin/hipcc","-O3","-std=c++17","-fPIC","-shared","--offload-arch=gfx950","-ffp-contract=off","-fno-fast-math",
  "-fhip-fp32-correctly-rounded-divide-sqrt","-DPBR_FAITHFUL_GAMMA_LO=0x1p-60f","-I",os.path.join(ROOT,"physically_based_renderer_amd","csrc"),
  os.path.join(ROOT,"tests","hip","gamma_probe.hip"),"-o",so,"-lpthread"],check=True)
L=ctypes.CDLL(so)
lo,hi=-60,-1
out=(ctypes.c_double*(hi-lo+1))()
assert L.probe_gamma(lo,hi,out)==0
for e in range(lo,hi+1): print(f"binade 2^{e}: max_rel {out[e-lo]:.4g}", flush=True)
