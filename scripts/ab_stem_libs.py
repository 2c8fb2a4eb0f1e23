"""A/B of the fused stem (stem_conv_kernel + the BatchNorm finalize + the vertical pool pass)
between builds (scripts/build_variants.sh): every library in AB_LIBS runs config 5's stem --
maxpool(relu(bn1(conv1(x)))) of 1,507 224 x 224 bf16 instances (PROBE_K to change the count),
torchvision ResNet-18 shapes, batch statistics -- in its own process (MCGMIL_LIB), reports the
time per call, and the parent checks the outputs bitwise against the first library.
An entry may add environment settings for its process: lib.so+NAME=VALUE.
Usage: AB_LIBS=abvar/base.so,abvar/split2.so python scripts/ab_stem_libs.py"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out_dir):
    import torch
    import torch.nn as nn
    sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
    from mcgmil.features import stem
    from mcgmil.resnet import deactivate_batchnorm
    dev = torch.device("cuda", 0)
    k = int(os.environ.get("PROBE_K", "1507"))
    torch.manual_seed(3)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    bn = nn.BatchNorm2d(64).to(dev).eval()
    with torch.no_grad():
        bn.weight.uniform_(-1.0, 1.0)      # both signs: the pool takes the minimum where gamma < 0
        bn.bias.uniform_(-0.5, 0.5)
    deactivate_batchnorm(bn)
    pool = nn.MaxPool2d(3, 2, 1)
    x = torch.randn(k, 3, 224, 224, device=dev).bfloat16()
    with torch.no_grad():
        y = stem(conv, bn, True, pool, x)
        for _ in range(3):
            stem(conv, bn, True, pool, x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            stem(conv, bn, True, pool, x)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    v = y.contiguous().view(torch.int16).flatten().to(torch.int64)
    wgt = torch.arange(v.numel(), device=dev, dtype=torch.int64) % 7919 + 1
    torch.save({"head": v[:4096].cpu(), "sum": v.sum().cpu(), "wsum": (v * wgt).sum().cpu()},
               os.path.join(out_dir, "stem.pt"))
    del v, wgt
    print(json.dumps({"lib": os.environ["AB_TAG"], "k": k, "stem_ms": round(ms, 4)}), flush=True)


def main():
    if os.environ.get("AB_CHILD"):
        return child(os.environ["AB_CHILD"])
    import torch
    specs = [q for q in os.environ["AB_LIBS"].split(",") if q]
    dirs = []
    for spec in specs:
        lib, *envs = spec.split("+")
        d = tempfile.mkdtemp(prefix="abstem_")
        env = dict(os.environ, MCGMIL_LIB=os.path.abspath(lib), AB_CHILD=d, AB_TAG=spec)
        env.update(e.split("=", 1) for e in envs)
        rc = subprocess.call([sys.executable, os.path.abspath(__file__)], env=env)
        if rc != 0:
            print(json.dumps({"lib": spec, "rc": rc}))
            return rc
        dirs.append(d)
    ref = torch.load(os.path.join(dirs[0], "stem.pt"), weights_only=True)
    ok = True
    for d, spec in zip(dirs[1:], specs[1:]):
        b = torch.load(os.path.join(d, "stem.pt"), weights_only=True)
        eq = all(torch.equal(b[q], ref[q]) for q in ("head", "sum", "wsum"))
        ok &= eq
        if not eq:
            print(json.dumps({"lib": spec, "bitwise": False}))
    print(json.dumps({"bitwise_equal_all": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
