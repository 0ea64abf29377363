"""Run np_pw2_probe on near-tie data and compare with NumPy (GPU box)."""
import os, subprocess
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.chdir(ROOT)
os.makedirs("gpurun_out", exist_ok=True)
for d in [2, 16, 64, 128, 200, 250]:
    rng = np.random.default_rng(d)
    X = (rng.standard_normal((300, d)) * 5).astype(np.float32)
    base = rng.standard_normal((8, d)) * 5
    C = np.concatenate([base, np.nextafter(base, np.inf), np.nextafter(base, -np.inf)])
    X.tofile("gpurun_out/px.bin")
    C.tofile("gpurun_out/pc.bin")
    subprocess.run(["./scripts/probes/np_pw2_probe", "gpurun_out/px.bin", "gpurun_out/pc.bin",
                    str(len(X)), str(len(C)), str(d)], check=True)
    S = np.fromfile("gpurun_out/pw2_sums.bin").reshape(len(X), len(C))
    diff = C[None] - X.astype(np.float64)[:, None]
    Sr = np.add.reduce(diff * diff, axis=-1)
    print(f"d={d}: lockstep sums differ from NumPy {(S != Sr).sum()}/{S.size}")
