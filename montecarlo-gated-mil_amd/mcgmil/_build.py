"""Build the in-tree HIP library libmcgmil.so for gfx950 (hipcc cross-compiles without a GPU).

The .so is written next to this file (git-ignored) so it travels to the GPU box with the repo
snapshot and is what the drop-in module loads.
"""
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(os.path.dirname(ROOT), "include")
LIB = os.path.join(PKG, "libmcgmil.so")
SOURCES = ["mcgmil.hip", "mcgmil_fused.hip", "mcgmil_image.hip", "mcgmil_bn.hip", "mcgmil_conv.hip", "mcgmil_stem.hip",
           "mcgmil_conv32.hip", "mcgmil_calib.hip"]
DEPS = ["mcgmil.hip", "mcgmil_fused.hip", "mcgmil_fused.h", "mcgmil_image.hip", "mcgmil_bn.hip", "mcgmil_conv.hip", "mcgmil_stem.hip",
        "mcgmil_conv32.hip", "mcgmil_calib.hip", "mcgmil_kernels.h",
        "mcgmil_device.h", "mcgmil_error.h", "mcgmil_gate_pp.h"]
ARCH = os.environ.get("MCGMIL_OFFLOAD_ARCH", "gfx950")
# No packed-fp32 VALU (v_pk_fma/mul/add_f32): with ROCm 7.2's compiler a packed write into the
# source VGPR of a just-issued v_rcp_f32 / v_exp_f32 gets no wait states, and on gfx950 the
# transcendental then sometimes reads the new value (nondeterministic low halves of the gate
# epilogue, found by scripts/probe_determinism.py). Scalar fp32 VALU is hazard-checked.
DEVICE_FLAGS = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
# Per-source flags. The MCDO gate kernels are scheduled with LLVM's max-ILP strategy: +3.0% on the
# bf16 separate-heads kernel and +1.1% shared, -1.8% on fp32 separate heads, measured in one process
# with scripts/probe_gate.py (MCGMIL_PROBE_LIBS; profiles/r01/probe_sched.log). The convolution
# and BatchNorm sources keep the default scheduler, and so does mcgmil_fused.hip: under max-ILP its
# tile loop spills (256 VGPRs + 64-220 B of scratch), with the default one it fits in 254.
SOURCE_FLAGS = {"mcgmil.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def _stale(out: str = LIB) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    if os.path.getmtime(os.path.abspath(__file__)) > t:      # build flags changed
        return True
    deps = [os.path.join(CSRC, d) for d in DEPS] + \
        [os.path.join(INCLUDE, h) for h in ("mcgmil.h", "mcgmil_image.h", "mcgmil_features.h", "mcgmil_calib.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=()) -> str:
    """Build libmcgmil.so (or, with defines such as MCGMIL_STAMPS, a diagnostic variant at
    `out`)."""
    if not force and not _stale(out):
        return out
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    tmp = out + ".tmp"
    objs, cmds = [], []
    for src in SOURCES:     # one object per source (per-source flags), then one shared library
        obj = f"{out}.{src}.o"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-c", "-fPIC", "-Wall", "-Werror",
               f"-I{INCLUDE}", "-o", obj] + DEVICE_FLAGS + SOURCE_FLAGS.get(src, []) + \
              [f"-D{d}" for d in defines] + [os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
        objs.append(obj)
    # the sources compile independently: in parallel (a few CPUs; each hipcc is single-threaded)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 1), 8))
    with ThreadPoolExecutor(jobs) as ex:
        for r in list(ex.map(lambda c: subprocess.run(c), cmds)):
            if r.returncode != 0:
                raise subprocess.CalledProcessError(r.returncode, r.args)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    for obj in objs:
        os.remove(obj)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force=True, verbose=True))
