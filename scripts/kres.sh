#!/bin/bash
# Per-kernel register / occupancy summary of a .hip file for gfx950.
f=${1:-ocean_model_arch_amd/csrc/sw_kernels.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off ${EXTRA:-} -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys,re
cur=None
for ln in sys.stdin:
    m=re.search(r"Function Name: (\S+)",ln)
    if m: cur=m.group(1); print("\n"+cur[:70],end=""); continue
    for k in ("VGPRs:","TotalSGPRs:","Occupancy \\[waves/SIMD\\]:","ScratchSize \\[bytes/lane\\]:","LDS Size \\[bytes/block\\]:"):
        m=re.search(k+r" (\d+)",ln)
        if m: print("  "+k.split()[0].rstrip(":")+"="+m.group(1),end="")
print()'
