#!/bin/bash
# Build an A/B twin of the library: the current objects with one source taken from a git revision.
#   bash scripts/ab_lib.sh <rev> <csrc file> <out.so>     e.g. HEAD esmstereo_amd/csrc/conv_small.hip
# Run a GPU script against it with ESM_LIB=<out.so> (esmstereo_amd/_lib.py).
set -e
rev=$1; src=$2; out=$3
cd "$(dirname "$0")/.."
tmp=esmstereo_amd/_abtmp  # same depth as csrc/: the sources include "../../include/..."
rm -rf "$tmp"; mkdir -p "$tmp"
git show "$rev:$src" > "$tmp/$(basename "$src")"
cp esmstereo_amd/csrc/*.h "$tmp/"
hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result \
    -c "$tmp/$(basename "$src")" -o "$tmp/ab.o"
base=$(basename "$src" .hip)
objs=$(ls esmstereo_amd/_build/*.o | grep -v "/$base.o$")
mkdir -p "$(dirname "$out")"
hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs "$tmp/ab.o"
rm -rf "$tmp"
echo "built $out ($src at $rev)"
