#!/bin/bash
# VGPR / SGPR / scratch / LDS of the one-pass march kernels in a built library (code object metadata):
# scripts/kernel_resources.sh [lib.so] [symbol regex]
set -eu
LIB=${1:-ocean_model_arch_amd/libocn_sw.so}
PAT=${2:-MarchStep}
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$LIB" "$T/fb.bin"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fb.bin" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/co.o"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/co.o" | python3 -c '
import sys, re
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split("\n  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or not pat.search(name.group(1)): continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    print(g("vgpr_count"), g("sgpr_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size"), name.group(1))
' "$PAT"
rm -rf "$T"
