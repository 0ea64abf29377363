"""Per-MFMA-gap instruction mix of the loop holding the most MFMAs (see
asm_loop.py): one line per MFMA with the counts of VALU / DS / VMEM / waits
issued after it, and the instructions after the last MFMA (the serial tail).
usage: asm_gaps.py file.s kernel_substring"""
import collections
import re
import subprocess
import sys

out = subprocess.run([sys.executable, __file__.replace("asm_gaps.py", "asm_loop.py"), sys.argv[1], sys.argv[2], "--text"],
                     capture_output=True, text=True, check=True).stdout.split("\n")
loop = [l.strip() for l in out if l and not l.startswith(" ") and not l.startswith("loop at")]
gaps = [collections.Counter()]
for l in loop:
    op = l.split()[0]
    if op.startswith("v_mfma"):
        gaps.append(collections.Counter())
        continue
    if op.endswith(":"):
        continue
    kind = ("ds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "scratch_")) else
            "wait" if op.startswith("s_waitcnt") else "nop" if op.startswith("s_nop") else
            "salu" if op.startswith("s_") else "valu")
    gaps[-1][kind] += 1
    if op.startswith("s_waitcnt"):
        gaps[-1]["w:" + l.split(None, 1)[1]] += 1
print("gap  valu  ds vmem salu nop waits")
for i, g in enumerate(gaps):
    w = " ".join(k[2:] for k in g if k.startswith("w:"))
    print(f"{i:3d} {g['valu']:5d} {g['ds']:3d} {g['vmem']:4d} {g['salu']:4d} {g['nop']:3d} {w}")
tot = sum(gaps[1:-1], collections.Counter())
print("in region:", dict((k, v) for k, v in tot.items() if not k.startswith("w:")))
print("head:", dict((k, v) for k, v in gaps[0].items() if not k.startswith("w:")),
      "tail:", dict((k, v) for k, v in gaps[-1].items() if not k.startswith("w:")))
