#!/bin/bash
# Host-side AddressSanitizer build of the C ABI and its check driver (tests/asan/abi_check.cpp).
# Only the host half of each translation unit is instrumented (-Xarch_host); device code is built
# as usual and never runs: the driver refuses to start when a GPU is visible.  CPU container only.
# Usage: bash scripts/asan_host.sh [iterations]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=build_asan
mkdir -p $OUT
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS=(-O1 -g -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude -Xarch_host -fsanitize=address
       -Xarch_host -fno-omit-frame-pointer)
pids=()
for src in esmstereo_amd/csrc/*.hip; do
    obj=$OUT/$(basename "${src%.hip}").o
    if [ ! -f "$obj" ] || [ -n "$(find esmstereo_amd/csrc include -newer "$obj" -name '*.h*' -print -quit)" ]; then
        extra=()
        case "$(basename "$src")" in volumes.hip|regression.hip) extra=(-ffp-contract=off) ;; esac
        "$HIPCC" "${FLAGS[@]}" "${extra[@]}" -c "$src" -o "$obj" &
        pids+=($!)
        if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
    fi
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" "${FLAGS[@]}" -c tests/asan/abi_check.cpp -o $OUT/abi_check.o
"$HIPCC" -fsanitize=address -fno-gpu-sanitize $OUT/*.o -o $OUT/abi_check
ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1 $OUT/abi_check "${1:-4000}"
