"""Where does the bf16 backbone's feature drift enter? A CPU emulation (round-3 verdict item 4).

The HIP bf16 backbone (mcgmil_conv.hip / mcgmil_bn.hip) takes bf16 operands, accumulates in fp32,
takes the BatchNorm batch statistics from the fp32 accumulators and stores every activation as
bf16. This script emulates exactly that storage rounding on torch CPU (fp32 convolutions on
bf16-rounded operands; rounding points switchable) on a random-init ResNet-18 with bag batch-stats
BN (reference infer.py:105-109) and reports the feature nrel against the all-fp32 network, per
variant:

  bf16          every stored activation rounded (the product path)
  fp32_last     the last block's output (BN2 + residual + ReLU) kept fp32 before the average pool
  fp32_layer4   all of layer 4's stored activations kept fp32
  fp32_stem     the stem's stored activations (conv output, BN + max-pool) kept fp32
  w_only        only the weights and the network input rounded; all activations fp32
  weights       only the weights rounded
  input         only the network input rounded

Usage: python scripts/probe_drift_cpu.py [instances] (default 48).
"""
import sys

import torch
import torch.nn.functional as F


def rb(x):
    return x.to(torch.bfloat16).to(torch.float32)


def bn(x, g, b):
    # batch statistics over the bag (training-mode BN, biased variance), fp32 as the HIP epilogue
    m = x.mean(dim=(0, 2, 3), keepdim=True)
    v = x.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    return (x - m) * torch.rsqrt(v + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def make_params(seed):
    g = torch.Generator().manual_seed(seed)

    def conv(o, i, k):
        fan_out = o * k * k
        return torch.randn(o, i, k, k, generator=g) * (2.0 / fan_out) ** 0.5

    def bnp(c):
        return (1.0 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g))

    P = {"stem": conv(64, 3, 7), "stem_bn": bnp(64), "layers": []}
    inp = 64
    for planes, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        blocks = []
        for bi in range(2):
            s = stride if bi == 0 else 1
            blk = {"c1": conv(planes, inp, 3), "b1": bnp(planes), "c2": conv(planes, planes, 3),
                   "b2": bnp(planes), "s": s, "down": None}
            if s != 1 or inp != planes:
                blk["down"] = (conv(planes, inp, 1), bnp(planes))
            blocks.append(blk)
            inp = planes
        P["layers"].append(blocks)
    return P


def forward(P, x, mode):
    """mode: 'fp32' or one of the bf16 variants in the module docstring."""
    if mode == "fp32":
        r = lambda t, where: t                                    # noqa: E731
    else:
        def r(t, where):
            if mode == "w_only" and where not in ("w", "in"):
                return t
            if mode == "weights" and where != "w":
                return t
            if mode == "input" and where != "in":
                return t
            if mode == "fp32_last" and where == "last":
                return t
            if mode == "fp32_layer4" and where in ("l4", "last"):
                return t
            if mode == "fp32_stem" and where == "stem":
                return t
            return rb(t)
    y = F.conv2d(r(x, "in"), r(P["stem"], "w"), stride=2, padding=3)
    y = r(y, "stem")                                              # stored conv output
    y = F.max_pool2d(F.relu(bn(y, *P["stem_bn"])), 3, 2, 1)
    y = r(y, "stem")
    for li, blocks in enumerate(P["layers"]):
        tag = "l4" if li == 3 else "act"
        for bi, blk in enumerate(blocks):
            last = li == 3 and bi == len(blocks) - 1
            idt = y
            if blk["down"] is not None:
                w, (g, b) = blk["down"]
                idt = r(F.conv2d(y, r(w, "w"), stride=blk["s"]), tag)
                idt = r(bn(idt, g, b), tag)
            h = r(F.conv2d(y, r(blk["c1"], "w"), stride=blk["s"], padding=1), tag)
            h = r(F.relu(bn(h, *blk["b1"])), tag)
            h = r(F.conv2d(h, r(blk["c2"], "w"), padding=1), tag)
            y = F.relu(bn(h, *blk["b2"]) + idt)
            y = r(y, "last" if last else tag)
    return y.mean(dim=(2, 3))                                     # the average pool, fp32


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    torch.manual_seed(0)
    P = make_params(1)
    # image-like instances: smooth positive patches, normalised as the pipeline does
    x = torch.rand(n, 3, 28, 28)
    x = F.interpolate(x, size=(224, 224), mode="bilinear", align_corners=False)
    x = (x - 0.5) / 0.25
    with torch.no_grad():
        ref = forward(P, x, "fp32")
        print(f"{n} instances, features |max| {ref.abs().max():.3f}")
        for mode in ("bf16", "fp32_last", "fp32_layer4", "fp32_stem", "w_only", "weights", "input"):
            f = forward(P, x, mode)
            nrel = float((f - ref).abs().max() / ref.abs().max())
            print(f"{mode:12s} feature nrel vs fp32: {nrel:.3e}", flush=True)


if __name__ == "__main__":
    main()
