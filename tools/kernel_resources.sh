#!/usr/bin/env bash
# Kernel register / LDS / scratch usage of a hipcc-built object or shared
# library (gfx950 code object metadata): tools/kernel_resources.sh OBJ [REGEX]
# Prints one line per kernel: vgpr agpr sgpr lds scratch name.
set -euo pipefail
obj=$1
pat=${2:-.}
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
LLVM=/opt/rocm/lib/llvm/bin
objcopy --dump-section .hip_fatbin="$tmp/fat.bin" "$obj" 2>/dev/null
target=$($LLVM/clang-offload-bundler --list --type=o --input="$tmp/fat.bin" | grep gfx950 | head -1)
$LLVM/clang-offload-bundler --unbundle --type=o --input="$tmp/fat.bin" --targets="$target" --output="$tmp/co.o"
$LLVM/llvm-readelf --notes "$tmp/co.o" | python3 -c '
import re, sys
pat = re.compile(sys.argv[1])
txt = sys.stdin.read()
for blk in txt.split("  - .agpr_count")[1:]:
    def f(k):
        m = re.search(r"\.%s:\s+(\S+)" % k, blk)
        return m.group(1) if m else "?"
    agpr = blk.split()[1]
    name = f("name")
    if pat.search(name):
        print(f("vgpr_count"), agpr, f("sgpr_count"), f("group_segment_fixed_size"),
              f("private_segment_fixed_size"), name)
' "$pat"
