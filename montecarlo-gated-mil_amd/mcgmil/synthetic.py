"""Seeded synthetic workload: bags of features and random-init head parameters.

No dataset or checkpoint can be fetched here, so the benchmark, the tests and the golden
fixtures all draw their inputs from this module. It is portable across machines (numpy PCG64),
so the committed fixtures store only outputs; inputs are regenerated from their seeds.

  H[n, l]   = |N(0, 1)|                      (post-ReLU/avg-pool ResNet-like features)
  weights   = U(-1/sqrt(fan_in), 1/sqrt(fan_in))  per nn.Linear, like torch's default init
State-dict keys follow the reference module (reference model.py:182-203).
"""
import numpy as np


def bag_features(seed: int, N: int, L: int = 512) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return np.abs(rng.standard_normal((N, L))).astype(np.float32)


def _linear(rng, out_f, in_f, bias=True):
    bound = 1.0 / np.sqrt(in_f)
    w = rng.uniform(-bound, bound, size=(out_f, in_f)).astype(np.float32)
    b = rng.uniform(-bound, bound, size=(out_f,)).astype(np.float32) if bias else None
    return w, b


def head_state_dict(seed: int, L: int = 512, D: int = 128, C: int = 2, shared: bool = False):
    """Parameters of the MIL head with the reference's state-dict key names."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    G = 1 if shared else C
    for g in range(G):
        pre_v = "attention_V.0" if shared else f"attention_V.{g}.0"
        pre_u = "attention_U.0" if shared else f"attention_U.{g}.0"
        w, b = _linear(rng, D, L)
        sd[pre_v + ".weight"], sd[pre_v + ".bias"] = w, b
        w, b = _linear(rng, D, L)
        sd[pre_u + ".weight"], sd[pre_u + ".bias"] = w, b
    for c in range(C):
        w, b = _linear(rng, 1, D)
        sd[f"attention_weights.{c}.weight"], sd[f"attention_weights.{c}.bias"] = w, b
    for c in range(C):
        w, _ = _linear(rng, 1, L, bias=False)
        sd[f"classifiers.{c}.weight"] = w
    return sd


def head_arrays(sd, C: int, shared: bool):
    """Stacked arrays (Wv[G,D,L], bv[G,D], Wu, bu, wa[C,D], ba[C], wk[C,L]) from a state dict."""
    G = 1 if shared else C
    def key(kind, g):
        return f"attention_{kind}.0" if shared else f"attention_{kind}.{g}.0"
    Wv = np.stack([sd[key("V", g) + ".weight"] for g in range(G)])
    bv = np.stack([sd[key("V", g) + ".bias"] for g in range(G)])
    Wu = np.stack([sd[key("U", g) + ".weight"] for g in range(G)])
    bu = np.stack([sd[key("U", g) + ".bias"] for g in range(G)])
    wa = np.concatenate([sd[f"attention_weights.{c}.weight"] for c in range(C)], axis=0)
    ba = np.concatenate([sd[f"attention_weights.{c}.bias"] for c in range(C)], axis=0)
    wk = np.concatenate([sd[f"classifiers.{c}.weight"] for c in range(C)], axis=0)
    return dict(Wv=Wv, bv=bv, Wu=Wu, bu=bu, wa=wa, ba=ba, wk=wk)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even to bf16, returned as float32 (finite inputs only)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def round_state_dict_bf16(sd, keys=("attention_V", "attention_U", "classifiers")):
    """bf16-round the GEMM weights (the operands the bf16 kernel consumes in bf16)."""
    out = {}
    for k, v in sd.items():
        out[k] = bf16_round(v) if (k.startswith(keys) and k.endswith("weight")) else v
    return out
