#!/bin/bash
# Build an A/B twin of the library: the current objects with some sources recompiled under extra
# defines.   bash scripts/ab_define.sh "-DESM_STORE_AUX=16" "conv_wide.hip conv_small.hip" out.so
set -e
defs=$1; files=$2; out=$3
cd "$(dirname "$0")/.."
tmp=esmstereo_amd/_abtmp
rm -rf "$tmp"; mkdir -p "$tmp"
objs=$(ls esmstereo_amd/_build/*.o)
for f in $files; do
    b=$(basename "$f" .hip)
    hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result $defs -c "esmstereo_amd/csrc/$f" -o "$tmp/$b.o" &
    objs=$(echo "$objs" | grep -v "/$b.o$" || true)
done
wait
mkdir -p "$(dirname "$out")"
hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs $tmp/*.o
rm -rf "$tmp"
echo "built $out ($files with $defs)"
