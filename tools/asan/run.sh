#!/bin/bash
# CPU AddressSanitizer build of gridbin.hip's host code (device code as usual,
# -fsanitize only on the host side), linked into tools/asan/gridbin_host.cpp.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}/dfhip_asan
mkdir -p "$O"
HASH=$(python3 -c "import sys; sys.path.insert(0, '$R/single-stable-dreamfusion_amd'); import dfhip_build; print(hex(dfhip_build.abi_hash()))")
F="--offload-arch=gfx950 -O1 -g -std=c++17 -ffp-contract=off -I$R/include -DDFHIP_ABI_HASH=$HASH -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
for f in gridbin errors; do
    hipcc $F -c "$R/single-stable-dreamfusion_amd/csrc/$f.hip" -o "$O/$f.o"
done
hipcc $F -c "$R/tools/asan/gridbin_host.cpp" -o "$O/driver.o"
hipcc --offload-arch=gfx950 -fsanitize=address "$O/driver.o" "$O/gridbin.o" "$O/errors.o" -o "$O/gridbin_host"
ASAN_OPTIONS=detect_leaks=0 "$O/gridbin_host"
