#!/usr/bin/env python3
"""Where a kernel's spills are: the 'Folded Spill' / 'Folded Reload' scratch instructions of
one function in an LLVM AMDGPU assembly file, counted by loop depth (from LLVM's block
comments) -- spills at depth 0 run once per launch, at depth >= 1 in the substep loop.
    python scripts/spill_map.py k.s 'k_step_quad<0, float>'"""
import re
import subprocess
import sys

src, want = sys.argv[1], sys.argv[2]
cur = None
depth = 0
out = {}
for line in open(src):
    m = re.match(r"^(_Z\S+):", line)
    if m:
        d = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = d if d.startswith("void " + want) or d.startswith(want) else None
        depth = 0
        continue
    if cur is None:
        continue
    if line.startswith(".Lfunc_end"):
        cur = None
        continue
    if re.match(r"^(\.LBB|; %bb)", line) or "; %bb." in line:
        m2 = re.search(r"Depth=(\d+)", line)
        depth = int(m2.group(1)) if m2 else 0
    t = line.strip()
    kind = "spill" if "Folded Spill" in t else ("reload" if "Folded Reload" in t else None)
    if kind is None and (t.startswith("scratch_") or (t.startswith("buffer_") and "offen" in t)):
        kind = "private_" + ("store" if "store" in t else "load")
    if kind:
        out.setdefault(depth, {}).setdefault(kind, 0)
        out[depth][kind] += 1
for d in sorted(out):
    print(f"loop depth {d}: " + ", ".join(f"{k} {v}" for k, v in sorted(out[d].items())))
