import ctypes, subprocess, os, sys, time
os.makedirs('build', exist_ok=True)
subprocess.run(['/opt/rocm/bin/hipcc','--offload-arch=gfx950','-O3','-ffp-contract=off','-fhip-fp32-correctly-rounded-divide-sqrt','-fPIC','-shared','-o','build/fastdiv_probe.so','tests/hip/fastdiv_probe.hip'],check=True)
L=ctypes.CDLL('build/fastdiv_probe.so')
bad=ctypes.c_ulonglong(); first=ctypes.c_uint()
t=time.time(); rc=L.probe_recip(-64, 64, ctypes.byref(bad), ctypes.byref(first)); print('recip exhaustive e in [-64,64]: rc',rc,'bad',bad.value,'first',hex(first.value), '%.2fs'%(time.time()-t), flush=True)
rc=L.probe_recip(-126, 126, ctypes.byref(bad), ctypes.byref(first)); print('recip exhaustive e in [-126,126]: rc',rc,'bad',bad.value,'first',hex(first.value), flush=True)
ex=(ctypes.c_float*2)(); br=ctypes.c_ulonglong()
for (alo,ahi,blo,bhi) in [(-96,60,-60,60),(-30,30,-30,30),(-5,5,-5,5),(-100,-60,-10,10)]:
    t=time.time(); rc=L.probe_div(ctypes.c_ulonglong(12345+alo), 65536, 64, alo,ahi,blo,bhi, ctypes.byref(bad), ctypes.byref(br), ex)
    n=65536*256*64
    print(f'markstein a in 2^[{alo},{ahi}) b in 2^[{blo},{bhi}): rc {rc} samples {n:.3g} bad {bad.value} r1_not_rn {br.value} ex {ex[0]!r} {ex[1]!r} {time.time()-t:.1f}s', flush=True)
