#!/bin/bash
# Scratch (private segment) of the row-gate kernels per diagnostic define set: the asm LDS reads of
# the row-gate K loop are only safe in instantiations without spills (a spilled or copied register
# whose ds_read is still in flight would be overwritten when the data lands). Run before timing a
# variant on the GPU. Usage: bash scripts/check_rowgate_scratch.sh "" "-DMCGMIL_RG_DIAG=64" ...
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
i=0
for defs in "$@"; do
    for src in mcgmil.hip mcgmil_fused.hip; do
        extra=""
        [ "$src" = mcgmil.hip ] && extra="-mllvm -amdgpu-sched-strategy=max-ilp"
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S \
            -Xclang -target-feature -Xclang -packed-fp32-ops $extra $defs \
            -o "$tmp/$i.$src.s" montecarlo-gated-mil_amd/csrc/$src 2>/dev/null &
    done
    i=$((i + 1))
done
wait
i=0
for defs in "$@"; do
    for src in mcgmil.hip mcgmil_fused.hip; do
        python3 - "$tmp/$i.$src.s" "$defs" <<'PY'
import re, sys
s = open(sys.argv[1]).read()
out = []
for m in re.finditer(r"\.set (_ZN6mcgmil\d+rowgate_(?:scores|fused)_kernel\w*)\.private_seg_size, (\d+)", s):
    name = m.group(1)
    v = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", s)
    a = re.search(re.escape(name) + r"\.num_agpr, (\d+)", s)
    out.append(f"{name[15:60]}={m.group(2)}(v{v.group(1) if v else '?'},a{a.group(1) if a else '?'})")
print(repr(sys.argv[2]), " ".join(out))
PY
    done
    i=$((i + 1))
done
rm -rf "$tmp"
