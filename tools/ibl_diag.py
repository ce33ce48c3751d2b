"""Diagnostic: worst-differing pixels of the IBL pole/seam scene (tests/test_gpu_parity.py), with
their normals, GPU vs oracle values and bit distances."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from conftest import oracle_pass_from_constants  # noqa: E402
from oracle import oracle as O  # noqa: E402
from physically_based_renderer_amd import _native as N, envmap  # noqa: E402
from physically_based_renderer_amd.renderer import GBuffer, PassConstants, ShadingContext  # noqa: E402

rng = np.random.default_rng(77)
h, w = 64, 512
n_px = h * w
eps = (np.sign(rng.uniform(-1, 1, (2, n_px))) * 10.0 ** rng.uniform(-7, -1, (2, n_px)))
pole = np.stack([eps[0], np.where(rng.uniform(size=n_px) < 0.5, 1.0, -1.0), eps[1]])
seam = np.stack([-rng.uniform(0.05, 1, n_px), rng.uniform(-1, 1, n_px), eps[1]])
rand = rng.normal(size=(3, n_px))
pick = rng.integers(0, 3, n_px)
n = np.where(pick == 0, pole, np.where(pick == 1, seam, rand))
n = (n / np.linalg.norm(n, axis=0)).astype(np.float32)
n[:, :64] = np.array([[0.0, 1.0, 0.0], [0.0, -1.0, 0.0], [-1.0, 0.0, 0.0], [-1.0, 0.0, -0.0]] * 16, np.float32).T
p = np.zeros((15, h, w), np.float32)
p[0:3] = rng.uniform(-5, 5, (3, h, w))
p[3:6] = n.reshape(3, h, w)
p[6:15] = rng.uniform(0, 1, (9, h, w))
env = envmap.load_chelsea_stairs_env()
pc = PassConstants(ambient_mode=N.PBR_AMBIENT_IBL_DIFFUSE, eye_pos_w=(0.0, 0.0, -10.0))
with ShadingContext(0) as ctx:
    ctx.set_pass(pc)
    ctx.set_env_map(env)
    got = ctx.shade(GBuffer.from_host(p, torch.device("cuda", 0))).cpu().numpy()
ref = O.shade(list(p), oracle_pass_from_constants(pc), None, env, n_threads=8)
e = O.rel_err(got, ref)
ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
print("max_rel", e.max(), "bit_exact", O.bit_equal(got, ref).mean())
print("ulp histogram:", {int(k): int(v) for k, v in zip(*np.unique(np.minimum(ulp, 20), return_counts=True))})
for cat in range(3):
    m = (pick.reshape(h, w) == cat)[..., None] & np.ones((1, 1, 4), bool)
    print("category", ["pole", "seam", "random"][cat], "max_rel", e[m].max(), "bit_exact", (ulp[m] == 0).mean())
flat = np.argsort(e.max(axis=2).ravel())[::-1][:12]
for i in flat:
    y, x = divmod(int(i), w)
    print(f"px({y},{x}) N=({p[3, y, x]:.9g},{p[4, y, x]:.9g},{p[5, y, x]:.9g}) albedo={p[6:9, y, x]} "
          f"got={got[y, x]} ref={ref[y, x]} ulp={ulp[y, x]} rel={e[y, x].max():.3g}")
np.savez(os.path.join(ROOT, "gpurun_out", "ibl_diag.npz"), got=got, ref=ref)
