"""Instruction mix of a kernel's hottest loop in a hipcc -S listing.

    python tools/isa_loop.py <file.s> <kernel-symbol-substring>

Prints the kernel's VGPR / AGPR / spill counts and, for the basic block with
the most MFMAs (the main loop body), the count of each opcode."""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
starts = [m.start() for m in re.finditer(r"^(\S*" + re.escape(pat) + r"\S*):", s, re.M)]
if not starts:
    sys.exit(f"no kernel matching {pat}")
i = starts[0]
name = s[i:s.index(":", i)]
end = s.index(".Lfunc_end", i)
body = s[i:end]
meta = s[end:end + 20000]
for key in ("NumVgprs", "NumAgprs", "ScratchSize", "Occupancy"):
    m = re.search(r"; %s: (\S+)" % key, s[end:end + 4000])
    print(f"{key}: {m.group(1) if m else '?'}")
blocks = re.split(r"\n(?=\.LBB\S*:)", body)
best = max(blocks, key=lambda b: b.count("v_mfma"))
ops = collections.Counter(l.split()[0] for l in best.split("\n")
                          if l.strip() and not l.strip().startswith((";", ".")))
print(f"hottest block: {best.split(chr(10))[0][:60]} ({sum(ops.values())} instructions)")
for k, v in ops.most_common(40):
    print(f"  {v:5d} {k}")
