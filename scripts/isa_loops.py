#!/usr/bin/env python3
"""Loop census of one kernel in a hipcc -S listing: for every backward branch (loop
latch) the line span, instruction count and counts of VALU / SALU / spill traffic inside.
    python3 scripts/isa_loops.py file.s kernel_symbol_prefix"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and ":" in l and not l.startswith("\t"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end + 1]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < i:
            loops.append((labels[t], i, t))
def cnt(a, b):
    ins = [x.strip() for x in body[a:b + 1] if re.match(r"^\s+[a-z_]", x)]
    c = lambda p: sum(1 for x in ins if re.match(p, x))
    return len(ins), c(r"v_"), c(r"s_"), c(r"v_readlane|v_writelane"), c(r"scratch_"), c(r"ds_"), c(r"global_|buffer_")
print("%6s %6s %-12s %5s %5s %5s %5s %5s %5s %5s" % ("from", "to", "label", "ins", "valu", "salu", "rdln", "scr", "ds", "vmem"))
for a, b, t in sorted(loops, key=lambda x: (x[1] - x[0])):
    print("%6d %6d %-12s %5d %5d %5d %5d %5d %5d %5d" % ((a + start + 1, b + start + 1, t) + cnt(a, b)))
