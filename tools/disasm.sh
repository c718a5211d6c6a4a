#!/bin/bash
# Disassemble the gfx950 code object of one built object file.
#   tools/disasm.sh single-stable-dreamfusion_amd/build/gridencoder.o > /tmp/g.s
set -e
obj=$1
tmp=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$obj" "$tmp/fat.bin"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$tmp/fat.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$tmp/g.co"
/opt/rocm/lib/llvm/bin/llvm-objdump -d "$tmp/g.co"
rm -rf "$tmp"
