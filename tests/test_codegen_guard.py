"""Codegen properties DESIGN.md relies on, checked on the device assembly of mcgmil.hip and
mcgmil_fused.hip compiled with the library's own flags (mcgmil/_build.py; hipcc cross-compiles for gfx950 without a GPU):

* no packed-fp32 VALU (v_pk_fma/add/mul_f32) in any kernel -- the guard against the packed-write /
  transcendental-source hazard of DESIGN.md §5 ("A toolchain hazard found on the way");
* the two-kernel path's gate kernel (gate_pipe_kernel, bf16 operands, separate heads, Philox masks)
  and the shared-heads kernel fit the register file without scratch spills, at two waves per SIMD;
* so does the launch bench.py times (gate_fused_kernel, bf16 separate heads; mcgmil_fused.hip with
  its own flags), and it has no packed-fp32 VALU either;
* the halo convolutions of the config-5 backbone (conv3x3c64_kernel, conv3x3c64_ring_kernel,
  conv3x3_halo_kernel; every
  STATS / input-BN instantiation) have no scratch and fit 256 registers: they run one 8-wave
  workgroup per CU (two waves per SIMD), and a spill would put scratch traffic into the tap loop;
* the stem convolution (stem_conv_kernel) drains its LDS-DMA staging (s_waitcnt vmcnt(0)) right
  before every barrier that publishes a staged tile: its epilogue's LDS accesses are inline asm the
  compiler's wait-count pass cannot see, so nothing else would order them after the DMA.
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
HEADLINE = "_ZN6mcgmil16gate_pipe_kernelIDF16bLi2ELi2ELb0ELb1ELb0ELi8EEEvNS_10GateParamsE"   # RTV = 8: whole tiles
FUSED = "_ZN6mcgmil17gate_fused_kernelIDF16bLi2ELi2ELb1ELb0EEEvNS_10GateParamsE"
# the MCGMIL_CLOCK_PROBE instantiations (same loop code + two stamps) fit as well
HEADLINE_PROBE = HEADLINE.replace("Lb1ELb0EEEv", "Lb1ELb1EEEv")
FUSED_PROBE = FUSED.replace("Lb1ELb0EEEv", "Lb1ELb1EEEv")


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
    for sym in (HEADLINE, HEADLINE_PROBE):
        assert kernel_meta(device_asm, sym, "private_seg_size") == 0, sym
        assert kernel_meta(device_asm, sym, "num_vgpr") + \
            kernel_meta(device_asm, sym, "num_agpr") <= 256          # two waves per SIMD


def test_shared_heads_kernel_fits_without_spills(device_asm):
    # the dispatched shape for shared heads: RT = 8 row tiles, PPW = 2 pairs per wave, Philox masks
    syms = set(re.findall(r"\.set (_ZN6mcgmil14gate_pp_kernelIDF16bLi8ELi2ELi\dELb0ELb0E\w*)\.private_seg_size",
                          device_asm))
    assert syms, "no bf16 gate_pp_kernel instantiation found"
    for sym in syms:
        assert kernel_meta(device_asm, sym, "private_seg_size") == 0, sym


def test_fused_kernel_fits_without_spills(fused_asm):
    assert not re.findall(r"^\s*(v_pk_(?:fma|add|mul)_f32)\b", fused_asm, flags=re.M)
    for sym in (FUSED, FUSED_PROBE):
        assert kernel_meta(fused_asm, sym, "private_seg_size") == 0, sym
        assert kernel_meta(fused_asm, sym, "num_vgpr") + kernel_meta(fused_asm, sym, "num_agpr") <= 256, sym


@pytest.fixture(scope="module")
def conv_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "mcgmil_conv.hip")


def test_halo_conv_kernels_fit_without_spills(conv_asm):
    syms = set(re.findall(r"\.set (_ZN12_GLOBAL__N_1\d+conv3x3(?:c64|c64_ring|_halo)_kernelILb[01]ELb[01]E\w*)"
                          r"\.private_seg_size", conv_asm))
    # conv3x3c64 / conv3x3_halo x (STATS, XF), and the row-ring kernel's 4 at its default wave count
    assert len(syms) == 12, syms
    for sym in syms:
        assert kernel_meta(conv_asm, sym, "private_seg_size") == 0, sym
        # 512-thread workgroups, one per CU: two waves per SIMD, 256 registers each
        assert kernel_meta(conv_asm, sym, "num_vgpr") + kernel_meta(conv_asm, sym, "num_agpr") <= 256, sym


@pytest.fixture(scope="module")
def stem_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "mcgmil_stem.hip")


def _barrier_predecessors(text, sym):
    i = text.index(sym + ":")
    j = text.index(".Lfunc_end", i)
    lines = [x.split(";")[0].strip() for x in text[i:j].split("\n")]
    out = []
    for k, x in enumerate(lines):
        if x.startswith("s_barrier"):
            q = k - 1
            while q > 0 and (not lines[q] or lines[q].startswith(".")):
                q -= 1
            out.append(lines[q])
    return out


def test_stem_barriers_drain_the_staging_dma(stem_asm):
    syms = sorted(set(re.findall(r"^(_ZN12_GLOBAL__N_1\d+stem_conv_kernelILi\dELb([01])ELb[01]EEEvNS_8StemGeomE):",
                                 stem_asm, flags=re.M)))
    assert len(syms) == 32, len(syms)
    for sym, stats in syms:
        prev = _barrier_predecessors(stem_asm, sym)
        # the prologue's and the tile loop's barriers; STATS kernels end with one more barrier for
        # the statistics reduction, after the last DMA has been waited for
        staged = prev[:-1] if stats == "1" else prev
        assert len(staged) >= 2, (sym, prev)
        for x in staged:
            assert x.startswith("s_waitcnt") and "vmcnt(0)" in x, (sym, prev)
