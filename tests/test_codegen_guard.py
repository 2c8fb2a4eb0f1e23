"""Codegen properties DESIGN.md relies on, checked on the device assembly of mcgmil.hip compiled
with the library's own flags (mcgmil/_build.py; hipcc cross-compiles for gfx950 without a GPU):

* no packed-fp32 VALU (v_pk_fma/add/mul_f32) in any kernel -- the guard against the packed-write /
  transcendental-source hazard of DESIGN.md §5 ("A toolchain hazard found on the way");
* the headline kernel (gate_pipe_kernel, bf16 operands, separate heads, Philox masks) and the
  shared-heads kernel fit the register file without scratch spills, at two waves per SIMD.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))

HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
HEADLINE = "_ZN6mcgmil16gate_pipe_kernelIDF16bLi2ELi2ELb0ELb1EEEvNS_10GateParamsE"


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    from mcgmil import _build
    out = str(tmp_path_factory.mktemp("asm") / "mcgmil.s")
    cmd = [HIPCC, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", f"-I{_build.INCLUDE}",
           "--cuda-device-only", "-S", "-o", out] + _build.DEVICE_FLAGS + \
        _build.SOURCE_FLAGS.get("mcgmil.hip", []) + [os.path.join(_build.CSRC, "mcgmil.hip")]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        pytest.fail("hipcc -S of mcgmil.hip took more than 900 s")
    if r.returncode != 0:
        pytest.fail(f"hipcc -S of mcgmil.hip failed ({r.returncode}):\n{r.stderr[-4000:]}")
    with open(out) as f:
        text = f.read()
    shutil.rmtree(os.path.dirname(out), ignore_errors=True)
    return text


def kernel_meta(text, sym, key):
    m = re.search(rf"\.set {re.escape(sym)}\.{key}, (\d+)", text)
    assert m, (sym, key)
    return int(m.group(1))


def test_no_packed_fp32_valu(device_asm):
    found = re.findall(r"^\s*(v_pk_(?:fma|add|mul)_f32)\b", device_asm, flags=re.M)
    assert not found, f"{len(found)} packed-fp32 instructions (hazard of DESIGN.md §5)"


def test_headline_kernel_fits_without_spills(device_asm):
    assert kernel_meta(device_asm, HEADLINE, "private_seg_size") == 0
    assert kernel_meta(device_asm, HEADLINE, "num_vgpr") + \
        kernel_meta(device_asm, HEADLINE, "num_agpr") <= 256        # two waves per SIMD


def test_shared_heads_kernel_fits_without_spills(device_asm):
    # the dispatched shape for shared heads: RT = 8 row tiles, PPW = 2 pairs per wave, Philox masks
    syms = set(re.findall(r"\.set (_ZN6mcgmil14gate_pp_kernelIDF16bLi8ELi2ELi\dELb0ELb0E\w*)\.private_seg_size",
                          device_asm))
    assert syms, "no bf16 gate_pp_kernel instantiation found"
    for sym in syms:
        assert kernel_meta(device_asm, sym, "private_seg_size") == 0, sym
