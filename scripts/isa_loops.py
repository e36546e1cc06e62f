#!/usr/bin/env python3
"""Per-loop census of one kernel in a `hipcc --cuda-device-only -S` listing: every basic
block is attributed to its innermost loop (LLVM's "Loop: Header=... Depth=..." block
comments); for each loop header: depth, instructions, VALU, SALU, spill traffic
(v_readlane/v_writelane, scratch), LDS and VMEM instructions of the blocks directly in it.
    python3 scripts/isa_loops.py file.s kernel_symbol_prefix"""
import re
import sys
from collections import defaultdict

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and ":" in l)
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
cur = ("<top>", 0)
stats = defaultdict(lambda: defaultdict(int))
for l in lines[start:end + 1]:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):.*?(?:Header=(BB\d+_\d+) Depth=(\d+))?\s*$", l)
    if m:
        if m.group(2):
            cur = (m.group(2), int(m.group(3)))
        elif "Loop Header" in l or "Parent Loop" in l:
            mm = re.search(r"Depth=(\d+)", l)
            name = m.group(1).lstrip(".L")
            cur = (name, int(mm.group(1)) if mm else 1)
        else:
            cur = ("<top>", 0)
        continue
    m = re.match(r"^\s+([a-z_][a-z0-9_]*)", l)
    if not m:
        continue
    op = m.group(1)
    s = stats[cur]
    s["ins"] += 1
    s["valu"] += op.startswith("v_")
    s["salu"] += op.startswith("s_")
    s["spill"] += op in ("v_readlane_b32", "v_writelane_b32") or op.startswith("scratch_")
    s["ds"] += op.startswith("ds_")
    s["vmem"] += op.startswith(("global_", "buffer_", "flat_"))
print("%-14s %5s %6s %6s %6s %6s %5s %5s" % ("loop", "depth", "ins", "valu", "salu", "spill", "ds", "vmem"))
for (h, d), s in sorted(stats.items(), key=lambda x: (-x[0][1], x[0][0])):
    print("%-14s %5d %6d %6d %6d %6d %5d %5d" % (h, d, s["ins"], s["valu"], s["salu"], s["spill"], s["ds"], s["vmem"]))
