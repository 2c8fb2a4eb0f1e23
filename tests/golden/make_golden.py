"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE module itself.

Runs only where the read-only reference checkout exists (/root/reference); it is never run on
the GPU box. The reference's `model.py` imports `torchvision.models` at import time
(reference model.py:5) but never calls torchvision after construction, so a constructor-only
stand-in module is placed in sys.modules (resnet18() -> a module whose forward flattens
[N,512,1,1] -> [N,512]); the model is built with pretrained=False (no weight download).
The extracted features H are fed as a [1, N, 512, 1, 1] "image" tensor.

Dropout masks: the reference's nn.Dropout layers (model.py:206-209) are swapped for a
ReplayDropout subclass that applies supplied keep-masks with torch's own rule
x * (keep * fp32(1/(1-p))); call order is feature_dropout, attention_dropouts.0, .1, ...
The masks are the build's Philox masks (oracle/philox_oracle.c), so the fixtures pin both
the oracle restatement (oracle/mcdo_ref.py) and, transitively, the HIP kernel.

Fixture contents: only metadata + outputs; inputs/weights are regenerated from seeds by
oracle/synthetic.py and masks by oracle/philox.py.

Usage:  python tests/golden/make_golden.py
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))

from oracle import philox  # noqa: E402
from mcgmil import synthetic  # noqa: E402


def _install_torchvision_standin():
    class _FlattenNet(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.Linear(512, 1000)

        def forward(self, x):
            return self.fc(torch.flatten(x, 1))

    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet18 = lambda weights=None: _FlattenNet()
    tv.models = tvm
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm


class ReplayDropout(nn.Dropout):
    """nn.Dropout subclass (so the reference's enable_dropout, model.py:268-271, still
    toggles it) that applies queued keep-masks instead of drawing from torch's RNG."""

    def __init__(self, p):
        super().__init__(p)
        self.queue = []

    def forward(self, x):
        if not self.training:
            return x
        keep = self.queue.pop(0)
        assert tuple(keep.shape) == tuple(x.shape), (keep.shape, x.shape)
        scale = torch.tensor(philox.dropout_scale(self.p), dtype=torch.float32).to(x.dtype)
        return x * (keep.to(x.dtype) * scale)


def build_reference(C, shared, sd, p_f, p_a, D=128):
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import model as ref_model  # the reference module (read-only checkout)
    m = ref_model.MultiHeadGatedAttentionMIL(num_classes=C, backbone="r18", pretrained=False,
                                             L=512, D=D, feature_dropout=p_f,
                                             attention_dropout=p_a, shared_attention=shared)
    m.feature_dropout = ReplayDropout(p_f)
    m.attention_dropouts = nn.ModuleList([ReplayDropout(p_a) for _ in range(C)])
    own = m.state_dict()
    load = {k: torch.from_numpy(np.asarray(v)).reshape(own[k].shape) for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(load, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith("feature_extractor") for k in missing), missing
    return m


def run_case(name, *, N, T, C=2, shared=False, p_f=0.1, p_a=0.1, D=128, L=512,
             h_seed, w_seed, mask_seed, bag_ctr=0, bf16=False, full_A=True, serial=False,
             forward=False):
    H = synthetic.bag_features(h_seed, N, L)
    sd = synthetic.head_state_dict(w_seed, L=L, D=D, C=C, shared=shared)
    if bf16:
        H = synthetic.bf16_round(H)
        sd = synthetic.round_state_dict_bf16(sd)
    m = build_reference(C, shared, sd, p_f, p_a, D=D)
    x = torch.from_numpy(H).view(1, N, L, 1, 1)
    meta = dict(N=N, T=T, C=C, L=L, D=D, shared=int(shared), p_f=p_f, p_a=p_a, h_seed=h_seed,
                w_seed=w_seed, mask_seed=mask_seed, bag_ctr=bag_ctr, bf16=int(bf16))
    out = {k: np.asarray(v) for k, v in meta.items()}
    if forward:
        m.eval()
        with torch.no_grad():
            Y, A, aux = m(x)
        assert aux is None
        out["Y"], out["A"] = Y.numpy(), A.numpy()
    else:
        keepF = torch.from_numpy(philox.feature_keep(mask_seed, bag_ctr, T, N, L, p_f))
        keepA = torch.from_numpy(philox.attention_keep(mask_seed, bag_ctr, T, C, N, p_a))
        if serial:
            m.feature_dropout.queue = [keepF[t].unsqueeze(0) for t in range(T)]
            for i in range(C):
                m.attention_dropouts[i].queue = [keepA[t, i].view(1, 1, N) for t in range(T)]
            Y, A = m.mc_inference_serial(x, N=T, device="cpu")
        else:
            m.feature_dropout.queue = [keepF.unsqueeze(1)]
            for i in range(C):
                shape = (T, 1, N) if shared else (T, 1, 1, N)
                m.attention_dropouts[i].queue = [keepA[:, i].reshape(shape)]
            Y, A = m.mc_inference(x, N=T, device="cpu")
        assert m.feature_dropout.queue == [] and all(d.queue == [] for d in m.attention_dropouts)
        Y, A = Y.detach(), A.detach()
        out["Y"] = Y.numpy()
        if full_A:
            out["A"] = A.numpy()
        else:
            out["A_first"], out["A_last"] = A[0].numpy(), A[-1].numpy()
        A2 = A[:, 0]
        out["A_mean"] = A2.mean(0).numpy()
        out["A_var"] = A2.var(0).numpy()
        out["P_mean"] = torch.softmax(Y, -1)[:, 0].mean(0).numpy()
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: Y{tuple(out['Y'].shape)} -> {os.path.getsize(path)} B")


def dump_head_keys():
    """State-dict keys/shapes of the reference head (the checkpoint ABI, model.py:182-209)."""
    import json
    keys = {}
    for shared in (True, False):
        sd = synthetic.head_state_dict(0, shared=shared)
        m = build_reference(2, shared, sd, 0.1, 0.1)
        keys["shared" if shared else "separate"] = {
            k: list(v.shape) for k, v in m.state_dict().items()
            if not k.startswith("feature_extractor")}
    with open(os.path.join(OUT, "reference_head_keys.json"), "w") as f:
        json.dump(keys, f, indent=1, sort_keys=True)


def torchvision_resnet_keys(depth):
    """State-dict keys/shapes of torchvision's resnet18/34 (BasicBlock; torchvision
    models/resnet.py ResNet._make_layer) with fc replaced by an Identity (reference
    model.py:179) and every BatchNorm's running statistics removed by deactivate_batchnorm
    (reference main.py:62 before training, infer.py:154 before loading): weight, bias and
    num_batches_tracked remain. torchvision is not installed here, so this enumerates the
    architecture; it is the backbone half of the checkpoint ABI the build commits to."""
    blocks = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3]}[depth]
    keys = {"conv1.weight": [64, 3, 7, 7]}

    def bn(prefix, c):
        keys.update({prefix + ".weight": [c], prefix + ".bias": [c], prefix + ".num_batches_tracked": []})
    bn("bn1", 64)
    inplanes = 64
    for li, (planes, nb) in enumerate(zip((64, 128, 256, 512), blocks), start=1):
        for j in range(nb):
            pre = f"layer{li}.{j}"
            keys[pre + ".conv1.weight"] = [planes, inplanes, 3, 3]
            bn(pre + ".bn1", planes)
            keys[pre + ".conv2.weight"] = [planes, planes, 3, 3]
            bn(pre + ".bn2", planes)
            if j == 0 and (li > 1):
                keys[pre + ".downsample.0.weight"] = [planes, inplanes, 1, 1]
                bn(pre + ".downsample.1", planes)
            inplanes = planes
    return keys


def dump_checkpoint_keys():
    """Full key/shape list of a reference checkpoint (main.py:92-94 torch.save of the module's
    state_dict): the head half from the reference module itself, the backbone half from
    torchvision_resnet_keys (under feature_extractor.)."""
    import json
    out = {}
    for depth in (18, 34):
        for shared in (False, True):
            sd = synthetic.head_state_dict(0, shared=shared)
            m = build_reference(2, shared, sd, 0.1, 0.1)
            head = {k: list(v.shape) for k, v in m.state_dict().items()
                    if not k.startswith("feature_extractor")}
            keys = {"feature_extractor." + k: v for k, v in torchvision_resnet_keys(depth).items()}
            keys.update(head)
            out[f"r{depth}_{'shared' if shared else 'separate'}"] = keys
    with open(os.path.join(OUT, "reference_checkpoint_keys.json"), "w") as f:
        json.dump(out, f, indent=1)


def p1_cases():
    """p_feat = 1: torch's Dropout zeroes every feature, so the gates see their biases alone and
    every logit of a class is the same constant wa_c . (tanh(bv) * sigmoid(bu)) + ba_c; the pooled
    embedding is 0 and Y equals the classifier bias. The attention is uniform only where p_att = 1
    as well (edge_N50_T3_sep_p1): with p_att = 0.1 (edge_N40_T3_shared_pf1) some of those constant
    logits are dropped to 0 and A is not uniform. The build's scale is 0, its threshold 65536."""
    run_case("edge_N50_T3_sep_p1", N=50, T=3, p_f=1.0, p_a=1.0, h_seed=31, w_seed=32, mask_seed=33)
    run_case("edge_N40_T3_shared_pf1", N=40, T=3, shared=True, p_f=1.0, p_a=0.1, h_seed=34,
             w_seed=35, mask_seed=36)


def main():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden.py needs the reference checkout at /root/reference")
    _install_torchvision_standin()
    torch.set_num_threads(8)
    only = set(sys.argv[1:])     # e.g. "big ckpt": regenerate just those groups
    if only:
        if "ckpt" in only:
            dump_checkpoint_keys()
        if "big" in only:
            big_cases()
        if "p1" in only:
            p1_cases()
        return
    dump_head_keys()
    dump_checkpoint_keys()
    # (1) small bags, T=1 and T=4, shared and separate
    for shared in (False, True):
        tag = "shared" if shared else "sep"
        run_case(f"small_N64_T1_{tag}", N=64, T=1, shared=shared, h_seed=1, w_seed=2, mask_seed=3)
        run_case(f"small_N64_T4_{tag}", N=64, T=4, shared=shared, h_seed=4, w_seed=5, mask_seed=6,
                 bag_ctr=7)
        run_case(f"serial_N64_T4_{tag}", N=64, T=4, shared=shared, h_seed=4, w_seed=5, mask_seed=6,
                 bag_ctr=7, serial=True)
        run_case(f"forward_N64_{tag}", N=64, T=1, shared=shared, h_seed=8, w_seed=9, mask_seed=0,
                 forward=True)
    # ragged / edge shapes
    run_case("edge_N1_T3_sep", N=1, T=3, h_seed=10, w_seed=11, mask_seed=12)
    run_case("edge_N37_T5_shared", N=37, T=5, shared=True, h_seed=13, w_seed=14, mask_seed=15)
    run_case("edge_N100_T7_sep_p05", N=100, T=7, p_f=0.5, p_a=0.5, h_seed=16, w_seed=17,
             mask_seed=18)
    run_case("edge_N200_T3_sep_p0", N=200, T=3, p_f=0.0, p_a=0.0, h_seed=19, w_seed=20,
             mask_seed=21)
    run_case("edge_N130_T2_C3_sep_D64", N=130, T=2, C=3, D=64, h_seed=22, w_seed=23, mask_seed=24)
    run_case("edge_N96_T2_C1_shared", N=96, T=2, C=1, shared=True, h_seed=25, w_seed=26,
             mask_seed=27)
    run_case("edge_N64_T2_sep_p09", N=64, T=2, p_f=0.9, p_a=0.9, h_seed=28, w_seed=29,
             mask_seed=30)
    p1_cases()
    # (2) config 2: N=512, T=30, fp32
    run_case("cfg2_N512_T30_sep", N=512, T=30, h_seed=42, w_seed=0, mask_seed=42, bag_ctr=0)
    run_case("cfg2_N512_T30_shared", N=512, T=30, shared=True, h_seed=42, w_seed=0,
             mask_seed=42, bag_ctr=0)
    run_case("forward_N512_sep", N=512, T=1, h_seed=42, w_seed=0, mask_seed=0, forward=True)
    # (3) config 3 shape in fp32, (4) the same with bf16-rounded H and GEMM weights
    run_case("cfg3_N2048_T100_sep", N=2048, T=100, h_seed=43, w_seed=0, mask_seed=42,
             bag_ctr=1, full_A=False)
    run_case("cfg3_N2048_T100_sep_bf16in", N=2048, T=100, h_seed=43, w_seed=0, mask_seed=42,
             bag_ctr=1, bf16=True, full_A=False)
    run_case("cfg3_N2048_T100_shared_bf16in", N=2048, T=100, shared=True, h_seed=43, w_seed=0,
             mask_seed=42, bag_ctr=1, bf16=True, full_A=False)
    big_cases()


def big_cases():
    """Bags above 4096 instances (softmax_pool_kernel's streaming branch): the reference's
    inference settings (config.yml:31,34: overlap 0.75) give up to ~5.8k tiles per image."""
    run_case("big_N5500_T4_sep", N=5500, T=4, h_seed=50, w_seed=51, mask_seed=52, bag_ctr=3)
    run_case("big_N4100_T3_shared", N=4100, T=3, shared=True, h_seed=53, w_seed=54, mask_seed=55,
             bag_ctr=9)


if __name__ == "__main__":
    main()
