#!/bin/bash
# Build an A/B variant of the kernel library: one source recompiled with extra
# defines, linked with the other objects of the last build().
#   bash tools/variant_lib.sh NAME SOURCE "-DFOO=1 ..."  -> lib/libdfhip_NAME.so
set -eu
cd "$(dirname "$0")/.."
P=single-stable-dreamfusion_amd
name=$1; src=$2; defs=$3
mkdir -p /tmp/dfhip_variants
obj=/tmp/dfhip_variants/${name}_$(basename "$src" .hip).o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc \
    -mcode-object-version=5 -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude $defs \
    -c $P/csrc/$src -o "$obj"
objs=$(ls $P/build/*.o | grep -v "/$(basename "$src" .hip).o$")
hipcc --offload-arch=gfx950 -shared -fPIC $objs "$obj" -o $P/lib/libdfhip_$name.so
echo $P/lib/libdfhip_$name.so
