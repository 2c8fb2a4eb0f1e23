"""A/B of the BatchNorm statistics pass (bn_partial_kernel + bn_finalize_kernel, the path of the
layer-3/4 convolutions, whose 256 x 256 tiles emit no statistics) between builds
(scripts/build_variants.sh). Every library in AB_LIBS runs batchnorm_coefficients on config 5's
layer-3 (1,507 x 256 x 14 x 14) and layer-4 (1,507 x 512 x 7 x 7) activations in its own process
(MCGMIL_LIB) and reports the time per call; the parent checks the coefficients bitwise against
the first library.
Usage: AB_LIBS=abvar/base.so,abvar/rows4.so python scripts/ab_bn_stats.py"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = [(1507, 256, 14), (1507, 512, 7)]


def child(out_dir):
    import torch
    import torch.nn as nn
    sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
    from mcgmil.features import batchnorm_coefficients
    from mcgmil.resnet import deactivate_batchnorm
    dev = torch.device("cuda", 0)
    lib = os.path.basename(os.environ["MCGMIL_LIB"])
    g = torch.Generator(device=dev).manual_seed(7)
    res = {}
    for n, c, hw in SHAPES:
        bn = nn.BatchNorm2d(c).to(dev).eval()
        deactivate_batchnorm(bn)
        x = (torch.randn(n, c, hw, hw, device=dev, generator=g) * 2 + 0.5).bfloat16()
        x = x.contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            ab = batchnorm_coefficients(x, bn)
            for _ in range(3):
                batchnorm_coefficients(x, bn)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 50
            e0.record()
            for _ in range(reps):
                batchnorm_coefficients(x, bn)
            e1.record()
            torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        res["%d_%d" % (c, hw)] = ab.cpu()
        print(json.dumps({"lib": lib, "C": c, "hw": hw, "us": round(us, 2),
                          "GBps": round(x.numel() * 2 / us / 1e3, 1)}), flush=True)
    torch.save(res, os.path.join(out_dir, "ab.pt"))


def main():
    if os.environ.get("AB_CHILD"):
        return child(os.environ["AB_CHILD"])
    import torch
    libs = [q for q in os.environ["AB_LIBS"].split(",") if q]
    dirs = []
    for lib in libs:
        d = tempfile.mkdtemp(prefix="abbn_")
        env = dict(os.environ, MCGMIL_LIB=os.path.abspath(lib), AB_CHILD=d)
        rc = subprocess.call([sys.executable, os.path.abspath(__file__)], env=env)
        if rc != 0:
            print(json.dumps({"lib": lib, "rc": rc}))
            return rc
        dirs.append(d)
    ref = torch.load(os.path.join(dirs[0], "ab.pt"), weights_only=True)
    ok = True
    for d, lib in zip(dirs[1:], libs[1:]):
        b = torch.load(os.path.join(d, "ab.pt"), weights_only=True)
        eq = all(torch.equal(b[k].view(torch.int32), ref[k].view(torch.int32)) for k in ref)
        ok &= eq
        if not eq:
            print(json.dumps({"lib": lib, "bitwise": False}))
    print(json.dumps({"bitwise_equal_all": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
