"""Host-side checks of the drop-in module (no kernel launches)."""
import json
import os

import pytest
import torch

from conftest import GOLDEN


def test_head_state_dict_keys_match_reference():
    """Reference checkpoints (model.py:182-209 parameter names/shapes) load strictly."""
    from mcgmil import MultiHeadGatedAttentionMIL
    ref = json.load(open(os.path.join(GOLDEN, "reference_head_keys.json")))
    for shared, tag in ((True, "shared"), (False, "separate")):
        m = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=shared)
        own = {k: list(v.shape) for k, v in m.state_dict().items()
               if not k.startswith("feature_extractor")}
        assert own == ref[tag]


def test_backbone_keys_follow_torchvision():
    from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm
    m = MultiHeadGatedAttentionMIL(pretrained=False)
    m.apply(deactivate_batchnorm)                     # infer.py:154
    keys = set(m.state_dict())
    for k in ("feature_extractor.conv1.weight", "feature_extractor.bn1.weight",
              "feature_extractor.layer1.0.conv1.weight", "feature_extractor.layer2.0.downsample.0.weight",
              "feature_extractor.layer4.1.bn2.bias", "feature_extractor.bn1.num_batches_tracked"):
        assert k in keys, k
    assert not any(k.endswith("running_mean") for k in keys)   # batch statistics, as infer.py
    assert not any(k.startswith("feature_extractor.fc") for k in keys)   # fc = Identity


def test_backbone_feature_shape_cpu():
    """The PyTorch-ROCm feeder (not the kernel) maps 3x224x224 instances to L=512 features."""
    from mcgmil import MultiHeadGatedAttentionMIL
    m = MultiHeadGatedAttentionMIL(pretrained=False)
    with torch.no_grad():
        H = m.extract_features(torch.randn(1, 3, 3, 64, 64))
    assert H.shape == (1, 3, 512)


def test_pretrained_warns_offline():
    from mcgmil import MultiHeadGatedAttentionMIL
    with pytest.warns(UserWarning):
        MultiHeadGatedAttentionMIL(pretrained=True, backbone="r34")


def test_no_cpu_path():
    from mcgmil import MultiHeadGatedAttentionMIL
    m = MultiHeadGatedAttentionMIL(pretrained=False)
    with pytest.raises(RuntimeError, match="HIP device"):
        m.mc_inference(torch.zeros(1, 2, 3, 32, 32), N=2, device="cpu")
    with pytest.raises(RuntimeError, match="HIP device"):
        m.mc_inference_features(torch.zeros(5, 512), T=2)
    m.train()
    with pytest.raises(NotImplementedError):
        m(torch.zeros(1, 2, 3, 32, 32))


def test_ops_reject_cpu_tensors():
    from mcgmil import ops
    head = ops.HeadTensors(*[torch.zeros(1, 1) for _ in range(7)])
    with pytest.raises(ValueError):
        ops.mcdo_forward(torch.zeros(4, 512), torch.zeros(2, dtype=torch.int32), head, 2,
                         p_feat=0.1, p_att=0.1, seed=0)


def test_bag_offsets_validation():
    from mcgmil import ops
    assert ops.bag_offsets_tensor([3, 0, 5], "cpu").tolist() == [0, 3, 3, 8]
    with pytest.raises(ValueError):
        ops.bag_offsets_tensor([0, 5, 3], "cpu", are_sizes=False)


def test_torch_library_ops_registered_with_fake_shapes():
    """The custom ops are registered; their fake kernels give the output shapes
    without touching a device, so graph captures can trace through them."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    from mcgmil import library  # noqa: F401
    assert hasattr(torch.ops.mcgmil, "mcdo_forward") and hasattr(torch.ops.mcgmil, "mcdo_forward_stats")
    R, L, D, C, G, T, B = 300, 512, 128, 2, 2, 7, 3
    with FakeTensorMode():
        H = torch.empty(R, L, dtype=torch.bfloat16)
        offs = torch.empty(B + 1, dtype=torch.int32)
        head = (torch.empty(G, D, L), torch.empty(G, D), torch.empty(G, D, L), torch.empty(G, D),
                torch.empty(C, D), torch.empty(C), torch.empty(C, L))
        Y, A = torch.ops.mcgmil.mcdo_forward(H, offs, *head, T, 0.1, 0.1, 5, 0, 0)
        Y2, Am, Av, Pm = torch.ops.mcgmil.mcdo_forward_stats(H, offs, *head, T, 0.1, 0.1, 5, 0, 0)
    assert tuple(Y.shape) == (B, T, C) and tuple(A.shape) == (T * C * R,) and A.dtype == torch.float32
    assert tuple(Y2.shape) == (B, T, C) and tuple(Am.shape) == tuple(Av.shape) == (C * R,)
    assert tuple(Pm.shape) == (B, C)


def test_torch_library_op_has_no_cpu_path():
    from mcgmil import library  # noqa: F401
    R, L, D, C = 8, 64, 16, 2
    head = (torch.zeros(C, D, L), torch.zeros(C, D), torch.zeros(C, D, L), torch.zeros(C, D),
            torch.zeros(C, D), torch.zeros(C), torch.zeros(C, L))
    with pytest.raises(ValueError, match="CUDA"):
        torch.ops.mcgmil.mcdo_forward(torch.zeros(R, L), torch.tensor([0, R], dtype=torch.int32),
                                      *head, 2, 0.1, 0.1, 1, 0, 0)


@pytest.mark.parametrize("cfg", ["r18_separate", "r18_shared", "r34_separate"])
def test_reference_checkpoint_loads_strictly(tmp_path, cfg):
    """A reference checkpoint (main.py:92-94: torch.save of the module's state_dict after
    deactivate_batchnorm, main.py:62) with every key the reference module has -- head keys taken
    from the reference itself, backbone keys torchvision's (tests/golden/make_golden.py
    dump_checkpoint_keys) -- goes through torch.save / torch.load(weights_only=True) and loads
    with strict=True into the drop-in module, as infer.py:154-159 does; every value lands."""
    from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm
    spec = json.load(open(os.path.join(GOLDEN, "reference_checkpoint_keys.json")))[cfg]
    g = torch.Generator().manual_seed(0)
    sd = {k: (torch.zeros((), dtype=torch.int64) if k.endswith("num_batches_tracked")
              else torch.randn(shape, generator=g)) for k, shape in spec.items()}
    path = tmp_path / "ckpt.pth"
    torch.save(sd, path)
    loaded = torch.load(path, map_location="cpu", weights_only=True)
    depth, att = cfg.split("_")
    # pretrained=False builds resnet18 whatever the backbone (reference model.py:177-178);
    # infer.py constructs with the default pretrained=True (offline here: random init + warning)
    with pytest.warns(UserWarning):
        m = MultiHeadGatedAttentionMIL(num_classes=2, backbone=depth, pretrained=True,
                                       shared_attention=(att == "shared"))
    m.apply(deactivate_batchnorm)                                 # infer.py:154
    assert {k: list(v.shape) for k, v in m.state_dict().items()} == spec
    m.load_state_dict(loaded, strict=True)                        # infer.py:159
    own = m.state_dict()
    for k, v in sd.items():
        assert torch.equal(own[k], v), k


@pytest.mark.parametrize("shared", [True, False])
def test_head_param_cache_sees_replaced_modules_and_parameters(shared):
    """_head_params (the per-bag caller's cached parameter list, model.py:182-203 order) follows a
    replaced Linear inside a container, a newly assigned Parameter and load_state_dict(assign=True);
    an unchanged module keeps the cached list."""
    import torch.nn as nn
    from mcgmil import MultiHeadGatedAttentionMIL
    m = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=shared)
    p0 = m._head_params()
    assert m._head_params() is p0                                    # hit: same list object
    new_w = nn.Parameter(torch.randn_like(m.classifiers[0].weight))
    m.classifiers[0].weight = new_w
    p1 = m._head_params()
    assert p1 is not p0 and any(p is new_w for p in p1)
    lin = nn.Linear(m.L, m.D)
    if shared:
        m.attention_V[0] = lin
    else:
        m.attention_V[1][0] = lin
    p2 = m._head_params()
    assert any(p is lin.weight for p in p2) and any(p is lin.bias for p in p2)
    sd = {k: v.clone() + 1 for k, v in m.state_dict().items() if not k.startswith("feature_extractor")}
    m.load_state_dict(sd, strict=False, assign=True)
    p3 = m._head_params()
    assert all(m2._parameters[n] is p for (m2, n), p in zip(m._head_slots(), p3))
    assert not any(p is q for p in p3 for q in p2)                   # every parameter was replaced
    assert len(p3) == len(p0)
