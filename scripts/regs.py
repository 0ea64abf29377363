"""Register / spill summary of kernels matching a pattern (hipcc resource remarks).
usage: python scripts/regs.py PATTERN [source.hip]"""
import re
import subprocess
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "k_"
src = sys.argv[2] if len(sys.argv) > 2 else "assignment--2-group7-distributed-k-means_amd/csrc/km_kernels.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
       "-mllvm", "-amdgpu-mfma-vgpr-form", "-c", src, "-o", "/tmp/regs_probe.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, out = None, {}
for l in err.splitlines():
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        out[cur] = {}
        continue
    m = re.search(r"remark:\s+([\w ]+?)(?: \[bytes/lane\]| \[waves/SIMD\])?: (\S+) \[", l)
    if m and cur:
        out[cur][m.group(1)] = m.group(2)
    if "error" in l:
        print(l)
for f, v in out.items():
    if pat in f:
        print(f"{f[:60]:60s} vgpr {v.get('VGPRs'):>4} agpr {v.get('AGPRs'):>4} spill {v.get('VGPRs Spill'):>3} "
              f"occ {v.get('Occupancy')}")
