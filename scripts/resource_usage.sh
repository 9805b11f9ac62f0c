#!/bin/bash
# Per-kernel register / scratch / occupancy of the step and reset kernels (device-only compile
# with -Rpass-analysis=kernel-resource-usage; ~3.5 min).  Extra hipcc flags as arguments:
#   bash scripts/resource_usage.sh [-DPOB_...]
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
  -mcode-object-version=5 --offload-device-only -c -Rpass-analysis=kernel-resource-usage "$@" \
  po-brax_amd/csrc/pob_kernels.hip -o $T/k.o > $T/ru.txt 2>&1
python3 - "$T/ru.txt" <<'PY'
import re, subprocess, sys
rows, cur = [], None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    d = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    if "k_step" in d or "k_reset" in d or "_ool" in d:
        d = d.split("(")[0]
        print(f"{d:<40} VGPR {r.get('VGPRs', 0):4d} AGPR {r.get('AGPRs', 0):4d} scratch {r.get('ScratchSize', 0):4d} B/lane "
              f"spillV {r.get('VGPRs Spill', 0):4d} occ {r.get('Occupancy', 0)}")
PY
rm -rf $T
