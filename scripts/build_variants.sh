#!/bin/bash
# Build A/B variants of libmcgmil.so (one per -D set), in parallel, into $VAR_OUT (default
# abvar/, git-ignored but shipped to the GPU box with the snapshot; build/ is gpurun-ignored).
# Usage: bash scripts/build_variants.sh "NAME:-DX=1 -DY=2" "NAME2:..." ...
#   A NAME of the form "name@REV" builds the sources of git revision REV instead of the tree.
set -e
OUT=${VAR_OUT:-abvar}
mkdir -p "$OUT"
rm -f "$OUT"/*.so "$OUT"/*.o
for spec in "$@"; do
    name=${spec%%:*}; defs=${spec#*:}
    src=montecarlo-gated-mil_amd/csrc; inc=include
    if [[ $name == *@* ]]; then
        rev=${name#*@}; name=${name%@*}
        tmp=$(mktemp -d)
        git archive "$rev" montecarlo-gated-mil_amd/csrc include | tar -x -C "$tmp"
        src=$tmp/montecarlo-gated-mil_amd/csrc; inc=$tmp/include
    fi
    # per source, as mcgmil/_build.py: the gate kernels (mcgmil.hip) with the max-ILP scheduler
    (
        objs=""
        srcs="mcgmil.hip mcgmil_fused.hip mcgmil_image.hip mcgmil_bn.hip mcgmil_conv.hip mcgmil_stem.hip mcgmil_conv32.hip mcgmil_calib.hip"
        [ -n "${GATE_ONLY:-}" ] && srcs="mcgmil.hip mcgmil_fused.hip"   # gate-kernel A/B: the MCDO entry points only
        for f in $srcs; do
            [ -f "$src/$f" ] || continue
            extra=""
            [ "$f" = mcgmil.hip ] && extra="${GATE_SCHED--mllvm -amdgpu-sched-strategy=max-ilp}"
            [ "$f" = mcgmil_fused.hip ] && extra="${FUSED_SCHED-}"
            nopk="-Xclang -target-feature -Xclang -packed-fp32-ops"
            [[ " $defs " == *" -DMCGMIL_PACKED=1 "* ]] && nopk=""   # packed-fp32 codegen on
            /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c -fPIC -I"$inc" \
                $nopk $extra $defs \
                -o "$OUT/$name.$f.o" "$src/$f" 2>&1 | grep -v packed-fp32-ops || true
            objs="$objs $OUT/$name.$f.o"
        done
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/$name.so" $objs
        rm -f $objs
    ) &
done
wait
ls "$OUT"
