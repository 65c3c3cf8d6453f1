#!/bin/bash
# Instruction streams of every kernel in a built library, addresses and branch offsets stripped:
# scripts/isa_dump.sh [lib.so] > out.txt -- two builds that should compile to the same machine code
# (e.g. before / after removing dead compile-time switches) give identical dumps.
set -eu
LIB=${1:-ocean_model_arch_amd/libocn_sw.so}
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$LIB" "$T/fb.bin"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fb.bin" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/co.o"
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 --no-show-raw-insn --no-leading-addr "$T/co.o" |
  sed -E '/^<.*>:$/b; s@//.*$@@; s@<[^>]*>@@g; s@(s_c?branch[a-z_0-9]*) .*@\1@; s@[[:space:]]+$@@' |
  grep -v -e '^$' -e 'file format'
rm -rf "$T"
