"""Verdict r05 item 5: would split-bf16 (hi + lo) weights on the layers where the drift enters
first cut config 5's bf16 uncertainty drift? CPU emulation on the rounding model of
scripts/probe_drift_cpu.py (bf16 operands, fp32 accumulation, bf16 stored activations, bag
batch-statistics BN), extended with:

  split weights   w = bf16(w) + bf16(w - bf16(w)): two MFMA passes per convolution (hi, lo) over
                  the same bf16 activations, accumulated in fp32 -- emulated exactly;
  split input     the network input as hi + lo (the patcher would write two bf16 planes);

and the MCDO head (oracle/mcdo_ref.py, model.py:280-316, T samples with the C Philox masks) on the
resulting features, so the drift is reported where the verdict measures it: A_mean / A_var nrel of
the head's outputs against the all-fp32 pipeline, next to the feature nrel.

Usage: python scripts/probe_split_bf16_drift.py [instances] [T]   (defaults 96, 100)
"""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "montecarlo-gated-mil_amd"), HERE]

from probe_drift_cpu import bn, make_params, rb  # noqa: E402


def split(t):
    hi = rb(t)
    return hi + rb(t - hi)


def forward(P, x, mode, wsplit=(), xsplit=False):
    """mode 'fp32' or 'bf16' (the product's rounding points); in bf16 mode the weights of the
    layers named in wsplit ('stem', 'l1'..'l4') are split hi + lo, and xsplit splits the input."""
    f32 = mode == "fp32"

    def r(t):
        return t if f32 else rb(t)

    def w(t, layer):
        if f32:
            return t
        return split(t) if layer in wsplit else rb(t)
    xin = x if f32 else (split(x) if xsplit else rb(x))
    y = r(F.conv2d(xin, w(P["stem"], "stem"), stride=2, padding=3))
    y = r(F.max_pool2d(F.relu(bn(y, *P["stem_bn"])), 3, 2, 1))
    for li, blocks in enumerate(P["layers"]):
        tag = f"l{li + 1}"
        for blk in blocks:
            idt = y
            if blk["down"] is not None:
                wd, (g, b) = blk["down"]
                idt = r(bn(r(F.conv2d(y, w(wd, tag), stride=blk["s"])), g, b))
            h = r(F.conv2d(y, w(blk["c1"], tag), stride=blk["s"], padding=1))
            h = r(F.relu(bn(h, *blk["b1"])))
            h = r(F.conv2d(h, w(blk["c2"], tag), padding=1))
            y = r(F.relu(bn(h, *blk["b2"]) + idt))
    return y.mean(dim=(2, 3))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    from mcgmil import synthetic
    from oracle import mcdo_ref
    torch.manual_seed(0)
    P = make_params(1)
    x = torch.rand(n, 3, 28, 28)
    x = F.interpolate(x, size=(224, 224), mode="bilinear", align_corners=False)
    x = (x - 0.5) / 0.25
    sd = synthetic.head_state_dict(0, C=2, shared=False)
    prm = mcdo_ref.HeadParams(synthetic.head_arrays(sd, 2, False))
    prm16 = mcdo_ref.HeadParams(synthetic.head_arrays(synthetic.round_state_dict_bf16(sd), 2, False))
    kF, kA = mcdo_ref.masks_for_bag(11, 0, T, n, 512, 2, 0.1, 0.1)

    def head(feat, p):
        Y, A = mcdo_ref.mc_inference(feat.numpy(), p, kF, kA, 0.1, 0.1)
        A = A[:, 0].double()                                           # [T, C, n]
        return A.mean(0), A.var(0)

    def nrel(a, b):
        return float((a - b).abs().max() / b.abs().max())
    with torch.no_grad():
        ref = forward(P, x, "fp32")
        m0, v0 = head(ref, prm)
        print(f"{n} instances, T={T}; head in fp32 on each variant's features (+ the bf16 head on them)")
        variants = [("bf16 (product)", (), False), ("split stem", ("stem",), False),
                    ("split stem+l1", ("stem", "l1"), False), ("split stem+l1+l2", ("stem", "l1", "l2"), False),
                    ("split all weights", ("stem", "l1", "l2", "l3", "l4"), False),
                    ("split input", (), True), ("split input+stem", ("stem",), True),
                    ("split input+stem+l1", ("stem", "l1"), True)]
        for name, ws, xs in variants:
            f = forward(P, x, "bf16", ws, xs)
            m, v = head(f, prm)
            fb = f.to(torch.bfloat16).float()
            mb, vb = head(fb, prm16)
            print(f"{name:22s} features {nrel(f, ref):.3e}  A_mean {nrel(m, m0):.3e}  A_var {nrel(v, v0):.3e}"
                  f"  | bf16 head: A_mean {nrel(mb, m0):.3e}  A_var {nrel(vb, v0):.3e}", flush=True)


if __name__ == "__main__":
    main()
