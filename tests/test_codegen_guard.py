"""Codegen properties DESIGN.md relies on, checked on the device assembly of mcgmil.hip and
mcgmil_fused.hip compiled with the library's own flags (mcgmil/_build.py; hipcc cross-compiles for gfx950 without a GPU):

* no packed-fp32 VALU (v_pk_fma/add/mul_f32) in any kernel -- the guard against the packed-write /
  transcendental-source hazard of DESIGN.md §5 ("A toolchain hazard found on the way");
* the two-kernel path's gate kernel (gate_pipe_kernel, bf16 operands, separate heads, Philox masks)
  and the shared-heads kernel fit the register file without scratch spills, at two waves per SIMD;
* so does the launch bench.py times (gate_fused_kernel, bf16 separate heads; mcgmil_fused.hip with
  its own flags), and it has no packed-fp32 VALU either;
* the halo convolutions of the config-5 backbone (conv3x3c64_kernel, conv3x3_halo_kernel; every
  STATS / input-BN instantiation) have no scratch: they run one 8-wave workgroup per CU at the
  register limit, and a spill would put scratch traffic into the tap loop.
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
FUSED = "_ZN6mcgmil17gate_fused_kernelIDF16bLi2ELi2ELb1EEEvNS_10GateParamsE"


def _asm(tmp_path_factory, source):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    from mcgmil import _build
    out = str(tmp_path_factory.mktemp("asm") / (source + ".s"))
    cmd = [HIPCC, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", f"-I{_build.INCLUDE}",
           "--cuda-device-only", "-S", "-o", out] + _build.DEVICE_FLAGS + \
        _build.SOURCE_FLAGS.get(source, []) + [os.path.join(_build.CSRC, source)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        pytest.fail(f"hipcc -S of {source} took more than 900 s")
    if r.returncode != 0:
        pytest.fail(f"hipcc -S of {source} failed ({r.returncode}):\n{r.stderr[-4000:]}")
    with open(out) as f:
        text = f.read()
    shutil.rmtree(os.path.dirname(out), ignore_errors=True)
    return text


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "mcgmil.hip")


@pytest.fixture(scope="module")
def fused_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "mcgmil_fused.hip")


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


def test_fused_kernel_fits_without_spills(fused_asm):
    assert not re.findall(r"^\s*(v_pk_(?:fma|add|mul)_f32)\b", fused_asm, flags=re.M)
    assert kernel_meta(fused_asm, FUSED, "private_seg_size") == 0
    assert kernel_meta(fused_asm, FUSED, "num_vgpr") + kernel_meta(fused_asm, FUSED, "num_agpr") <= 256


@pytest.fixture(scope="module")
def conv_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "mcgmil_conv.hip")


def test_halo_conv_kernels_fit_without_spills(conv_asm):
    syms = set(re.findall(r"\.set (_ZN12_GLOBAL__N_1\d+conv3x3(?:c64|_halo)_kernelILb[01]ELb[01]E\w*)\.private_seg_size",
                          conv_asm))
    assert len(syms) == 8, syms
    for sym in syms:
        assert kernel_meta(conv_asm, sym, "private_seg_size") == 0, sym
        assert kernel_meta(conv_asm, sym, "num_vgpr") + kernel_meta(conv_asm, sym, "num_agpr") <= 512, sym
