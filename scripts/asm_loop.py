"""Instruction histogram of the loop (label .. backward branch) holding the
most MFMAs in a kernel of a .s file.
usage: asm_loop.py file.s kernel_substring [--text]"""
import collections, re, sys
path, ksub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and ksub in l)
end = next((i for i in range(start + 1, len(lines)) if re.match(r"^_Z\S*:", lines[i]) or lines[i].startswith(".Lfunc_end")), len(lines))
body = lines[start:end]
labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\S+):", l)] if m}
best = None
for i, l in enumerate(body):
    m = re.search(r"s_cbranch\w*\s+(\.LBB\S+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        a = labels[m.group(1)]
        nm = sum("v_mfma" in x for x in body[a:i + 1])
        if nm and (best is None or i - a < best[2] - best[1]):
            best = (nm, a, i)
nm, a, b = best
loop = [l.strip() for l in body[a:b + 1] if l.strip() and not l.strip().startswith(";")]
ops = collections.Counter(l.split()[0] for l in loop if not l.endswith(":"))
print(f"loop at {body[a].split(':')[0]}: {sum(ops.values())} instructions, {nm} mfma")
for op, c in ops.most_common():
    print(f"  {c:4d} {op}")
if "--text" in sys.argv:
    print("\n".join(loop))
