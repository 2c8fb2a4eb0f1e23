#!/bin/bash
# Build A/B variants of libmcgmil.so into /tmp/mcgmil_var/ (one per -D set), in parallel.
# Usage: bash scripts/build_variants.sh "NAME:-DX=1 -DY=2" "NAME2:..." ...
set -e
mkdir -p /tmp/mcgmil_var
rm -f /tmp/mcgmil_var/*.so
for spec in "$@"; do
    name=${spec%%:*}; defs=${spec#*:}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Iinclude \
        -Xclang -target-feature -Xclang -packed-fp32-ops $defs \
        -o /tmp/mcgmil_var/$name.so montecarlo-gated-mil_amd/csrc/mcgmil.hip \
        montecarlo-gated-mil_amd/csrc/mcgmil_image.hip &
done
wait
ls /tmp/mcgmil_var
