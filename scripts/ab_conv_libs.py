"""A/B of convolution builds (scripts/build_variants.sh): every library named in AB_LIBS runs the
ResNet-18 layer-3/4 block convolutions of a config-5 bag (PROBE_K instances) in its own process
(MCGMIL_LIB), saves the outputs, and reports its per-layer time; the parent checks the outputs
bitwise against the first library. One JSON line per (library, layer) and one verdict line.
Usage: AB_LIBS=abvar_c/base.so,abvar_c/ph.so python scripts/ab_conv_libs.py
An entry may add environment settings for its process: lib.so+MCGMIL_CONV_SPLIT=0.
AB_SET=layer2 runs layer 2's 128 -> 128 3x3 convolution (conv3x3_halo_kernel) instead, plain, with
BatchNorm statistics, and with statistics + the input BatchNorm (the three launches of a config-5
image's layer 2)."""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (Cin, H, Cout, k, stride, pad, count in ResNet-18): the Cout % 256 == 0 layers
LAYERS = [(128, 28, 256, 3, 2, 1, 1), (128, 28, 256, 1, 2, 0, 1), (256, 14, 256, 3, 1, 1, 3),
          (256, 14, 512, 3, 2, 1, 1), (256, 14, 512, 1, 2, 0, 1), (512, 7, 512, 3, 1, 1, 3)]
# layer 2's halo launches per image: 1 with statistics, 2 with statistics + input BatchNorm
LAYERS2 = [(128, 28, 128, 3, 1, 1, 0, "plain"), (128, 28, 128, 3, 1, 1, 1, "stats"),
           (128, 28, 128, 3, 1, 1, 2, "xf")]


# layer 2's stride-2 convolutions from 64 channels: the 1x1 downsample (conv1x1_kernel) and the 3x3
# (conv_dma_kernel<256, 128>), with statistics as config 5 runs them, and plain
LAYERS_DOWN = [(64, 56, 128, 1, 2, 0, 1, "stats"), (64, 56, 128, 1, 2, 0, 0, "plain"),
               (64, 56, 128, 3, 2, 1, 1, "stats"), (64, 56, 128, 3, 2, 1, 0, "plain")]


def layers():
    if os.environ.get("AB_SET") == "layer2":
        return LAYERS2
    if os.environ.get("AB_SET") == "down":
        return LAYERS_DOWN
    return [t + ("plain",) for t in LAYERS]


def child(out_dir):
    import torch
    import torch.nn as nn
    sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
    from mcgmil.features import conv2d
    dev = torch.device("cuda", 0)
    K = int(os.environ.get("PROBE_K", "1507"))
    lib = os.path.basename(os.environ["MCGMIL_LIB"]) + os.environ.get("AB_TAG", "")
    tot = 0.0
    for li, (cin, h, cout, k, s, p, count, mode) in enumerate(layers()):
        g = torch.Generator(device=dev).manual_seed(100 + li)
        conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).eval()
        with torch.no_grad():
            conv.weight.copy_(torch.randn(conv.weight.shape, device=dev, generator=g) * 0.05)
        x = torch.randn(K, cin, h, h, device=dev, generator=g).relu_().bfloat16().contiguous(
            memory_format=torch.channels_last)
        conv = conv.to(memory_format=torch.channels_last)
        oh = (h + 2 * p - k) // s + 1
        flop = 2.0 * K * oh * oh * cout * cin * k * k
        kw = {}
        if mode != "plain":
            kw["stats"] = True
        if mode == "xf":
            ab = torch.stack([torch.rand(cin, device=dev, generator=g) + 0.5,
                              torch.randn(cin, device=dev, generator=g) * 0.1]).contiguous()
            kw["in_ab"] = ab
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            y = conv2d(conv, x, **kw)
            if mode != "plain":
                y = torch.cat([y[0].flatten(), y[1].flatten().view(torch.bfloat16)]) \
                    if y[1] is not None else y[0]
            torch.cuda.synchronize()
            reps = 10
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                conv2d(conv, x, **kw)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
        tot += ms * count
        torch.save(y.cpu(), os.path.join(out_dir, f"y{li}.pt"))
        print(json.dumps({"lib": lib, "cin": cin, "hw": h, "cout": cout, "k": k, "stride": s,
                          "mode": mode, "ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}), flush=True)
    key = {"layer2": "layer2_ms_per_image", "down": "downsample_ms_per_image"}.get(
        os.environ.get("AB_SET"), "layers_3_4_ms_per_image")
    print(json.dumps({"lib": lib, key: round(tot, 4)}), flush=True)


def main():
    if os.environ.get("AB_CHILD"):
        return child(os.environ["AB_CHILD"])
    import torch
    libs = [q for q in os.environ["AB_LIBS"].split(",") if q]
    dirs = []
    for lib in libs:
        d = tempfile.mkdtemp(prefix="abconv_")
        path, *sets = lib.split("+")
        env = dict(os.environ, MCGMIL_LIB=os.path.abspath(path), AB_CHILD=d,
                   AB_TAG="".join("+" + kv for kv in sets))
        env.update(kv.split("=", 1) for kv in sets)
        rc = subprocess.call([sys.executable, os.path.abspath(__file__)], env=env)
        if rc != 0:
            print(json.dumps({"lib": lib, "rc": rc}))
            return rc
        dirs.append(d)
    ok = True
    for li in range(len(layers())):
        ref = torch.load(os.path.join(dirs[0], f"y{li}.pt"), weights_only=True)
        for d, lib in zip(dirs[1:], libs[1:]):
            y = torch.load(os.path.join(d, f"y{li}.pt"), weights_only=True)
            eq = bool(torch.equal(y.view(torch.int16), ref.view(torch.int16)))   # bits (NaN-safe)
            ok &= eq
            if not eq:
                print(json.dumps({"layer": li, "lib": lib, "bitwise": False,
                                  "max_abs": float((y.float() - ref.float()).abs().max())}))
    print(json.dumps({"bitwise_equal_all": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
