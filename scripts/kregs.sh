#!/bin/bash
# Register counts / code size of the one-pass kernels in a built library (no GPU needed):
# scripts/kregs.sh [lib.so] [symbol pattern]
set -eu
LIB=${1:-ocean_model_arch_amd/libocn_sw.so}
PAT=${2:-MarchStepILb1ELb0ELb1ELb0ELb0E}
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$LIB" "$T/fb.bin"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fb.bin" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/co.o"
/opt/rocm/lib/llvm/bin/llvm-readelf -s "$T/co.o" | grep "$PAT" | grep -E "FUNC|num_vgpr|numbered_sgpr|private_seg" | awk '{print $2, $3, $8}' | sort -u
rm -rf "$T"
