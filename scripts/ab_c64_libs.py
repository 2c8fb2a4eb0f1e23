"""A/B of a ResNet 3x3 / stride-1 block convolution (default layer 1: 64 -> 64 at 56 x 56; AB_CIN=128
AB_HW=28 for layer 2) across library builds
(scripts/build_variants.sh): every library named in AB_LIBS runs the three forms config 5 uses --
plain, with the BatchNorm statistics epilogue, and with statistics + the input BatchNorm (in_ab) --
on PROBE_K instances in its own process (MCGMIL_LIB), saves the outputs and reports the time per
form; the parent checks the outputs bitwise against the first library (the statistics partials
follow each kernel's own lane order, so they are compared as per-channel totals).
Usage: AB_LIBS=abvar/ring.so,abvar/patch.so python scripts/ab_c64_libs.py"""
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
    from mcgmil.features import batchnorm_coefficients, conv2d, conv_input_bn
    from mcgmil.resnet import deactivate_batchnorm
    dev = torch.device("cuda", 0)
    K = int(os.environ.get("PROBE_K", "1507"))
    reps = int(os.environ.get("PROBE_REPS", "10"))
    lib = os.path.basename(os.environ["MCGMIL_LIB"])
    C = int(os.environ.get("AB_CIN", "64"))
    HW = int(os.environ.get("AB_HW", "56"))
    g = torch.Generator(device=dev).manual_seed(5)
    conv = nn.Conv2d(C, C, 3, 1, 1, bias=False).to(dev).eval()
    bn = nn.BatchNorm2d(C)
    deactivate_batchnorm(bn)
    bn = bn.to(dev).eval()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, device=dev, generator=g) * 0.06)
        bn.weight.copy_(torch.randn(C, device=dev, generator=g) * 0.5 + 1.0)
        bn.bias.copy_(torch.randn(C, device=dev, generator=g) * 0.3)
    conv = conv.to(memory_format=torch.channels_last)
    x = (torch.randn(K, C, HW, HW, device=dev, generator=g) + 0.3).bfloat16().contiguous(
        memory_format=torch.channels_last)
    flop = 2.0 * K * HW * HW * C * C * 9
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ab = batchnorm_coefficients(x, bn)
        forms = {"plain": lambda: conv2d(conv, x),
                 "stats": lambda: conv2d(conv, x, stats=True)}
        if conv_input_bn(conv, x):      # the layer's kernel takes the input BatchNorm
            forms["stats_inbn"] = lambda: conv2d(conv, x, stats=True, in_ab=ab, in_relu=True)
        for name, fn in forms.items():
            out = fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            y, part = out if isinstance(out, tuple) else (out, None)
            torch.save(y.cpu(), os.path.join(out_dir, f"{name}_y.pt"))
            if part is not None:
                tot = torch.stack([part[:, 0].sum(0), (part[:, 0] * part[:, 1]).sum(0)]).double().cpu()
                torch.save(tot, os.path.join(out_dir, f"{name}_s.pt"))
            print(json.dumps({"lib": lib, "form": name, "k": K, "cin": C, "hw": HW, "ms": round(ms, 4),
                              "tflops": round(flop / ms / 1e9, 1)}), flush=True)


def main():
    if os.environ.get("AB_CHILD"):
        return child(os.environ["AB_CHILD"])
    import torch
    libs = [q for q in os.environ["AB_LIBS"].split(",") if q]
    dirs = []
    for lib in libs:
        d = tempfile.mkdtemp(prefix="abc64_")
        env = dict(os.environ, MCGMIL_LIB=os.path.abspath(lib), AB_CHILD=d)
        rc = subprocess.call([sys.executable, os.path.abspath(__file__)], env=env)
        if rc != 0:
            print(json.dumps({"lib": lib, "rc": rc}))
            return rc
        dirs.append(d)
    ok = True
    for name in ("plain", "stats", "stats_inbn"):
        if not os.path.exists(os.path.join(dirs[0], f"{name}_y.pt")):
            continue
        ref = torch.load(os.path.join(dirs[0], f"{name}_y.pt"), weights_only=True)
        for d, lib in zip(dirs[1:], libs[1:]):
            y = torch.load(os.path.join(d, f"{name}_y.pt"), weights_only=True)
            eq = bool(torch.equal(y, ref))
            ok &= eq
            line = {"form": name, "lib": lib, "bitwise_y": eq}
            sp = os.path.join(d, f"{name}_s.pt")
            if os.path.exists(sp):
                s0 = torch.load(os.path.join(dirs[0], f"{name}_s.pt"), weights_only=True)
                s1 = torch.load(sp, weights_only=True)
                line["stats_sum_nrel"] = float(((s1 - s0).abs() / (s0.abs() + 1e-30)).max())
            print(json.dumps(line))
    print(json.dumps({"bitwise_equal_all": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
