#!/bin/bash
# Static instruction statistics of the step kernels' device code: per function (kernels and
# out-of-line device functions), the VALU instructions and the scratch (spill / private array)
# loads and stores in its own body.  Device-only compile to assembly (~3.5 min); extra hipcc
# flags as arguments.   bash scripts/asm_stats.sh [-D...] [| grep quad]
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
  -mcode-object-version=5 --offload-device-only -S "$@" po-brax_amd/csrc/pob_kernels.hip -o $T/k.s 2>/dev/null
python3 - "$T/k.s" <<'PY'
import re, subprocess, sys
cur, stats = None, {}
for line in open(sys.argv[1]):
    m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
    if m:
        cur = m.group(1)
        stats[cur] = [0, 0, 0]
        continue
    if cur is None:
        continue
    t = line.strip()
    if t.startswith("s_endpgm") or t.startswith(".Lfunc_end"):
        cur = None if t.startswith(".Lfunc_end") else cur
        continue
    if t.startswith("v_"):
        stats[cur][0] += 1
    if t.startswith("scratch_store") or (t.startswith("buffer_store") and "offen" in t):
        stats[cur][1] += 1
    if t.startswith("scratch_load") or (t.startswith("buffer_load") and "offen" in t):
        stats[cur][2] += 1
for name, (v, st, ld) in stats.items():
    d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip().split("(")[0]
    if "k_step" in d or "_ool" in d or "k_reset" in d:
        print(f"{d:<44} VALU {v:6d}  scratch stores {st:5d}  loads {ld:5d}")
PY
rm -rf $T
