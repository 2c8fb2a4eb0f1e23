#!/bin/bash
# Build tests/asan/capi_host_check against the library sources with AddressSanitizer and
# UndefinedBehaviorSanitizer on the HOST pass only (-Xarch_host; GPU sanitizers are not used).
# Usage: bash tests/asan/build.sh OUT_DIR   (prints the binary path)
set -euo pipefail
OUT=${1:?out dir}
REPO=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$OUT"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
HIPCC=${ROCM_PATH:-/opt/rocm}/bin/hipcc
objs=()
for f in mcgmil mcgmil_fused mcgmil_image mcgmil_bn mcgmil_conv mcgmil_stem; do
    "$HIPCC" --offload-arch=gfx950 -std=c++17 -O1 -I"$REPO/include" $SAN \
        -Xclang -target-feature -Xclang -packed-fp32-ops \
        -c "$REPO/montecarlo-gated-mil_amd/csrc/$f.hip" -o "$OUT/$f.o" 2>&1 | grep -v "packed-fp32-ops" || true
    objs+=("$OUT/$f.o")
done
"$HIPCC" --offload-arch=gfx950 -std=c++17 -O1 -I"$REPO/include" $SAN -x c++ \
    -c "$REPO/tests/asan/capi_host_check.cpp" -o "$OUT/capi_host_check.o"
"$HIPCC" --offload-arch=gfx950 $SAN "${objs[@]}" "$OUT/capi_host_check.o" -o "$OUT/capi_host_check"
echo "$OUT/capi_host_check"
