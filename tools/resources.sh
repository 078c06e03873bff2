#!/bin/bash
# tools/resources.sh — per-kernel VGPR / SGPR / scratch / occupancy of rtg_kernels.hip (gfx950)
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -Iinclude \
  -Iraytracing-practice_amd/csrc ${RES_DEFS:-} -c raytracing-practice_amd/csrc/rtg_kernels.hip -o /tmp/rtg_res.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); print(cur[:90], end=""); continue
    for key in ("VGPRs:", "SGPRs Spill:", "ScratchSize [bytes/lane]:", "Occupancy [waves/SIMD]:", "LDS Size [bytes/block]:"):
        if key in line:
            print("  %s %s" % (key.split()[0], line.split(key)[1].split()[0]), end="")
            if key.startswith("LDS"): print()
'
