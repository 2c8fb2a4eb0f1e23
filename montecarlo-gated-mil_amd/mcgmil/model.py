"""Drop-in MultiHeadGatedAttentionMIL whose MCDO inference path runs on the gfx950 kernels.

Mirrors the reference module xkuubix/MonteCarlo-Gated-MIL model.py:134-401:
  - same constructor keywords and defaults (model.py:135-145),
  - same submodule / parameter names and shapes, so reference checkpoints load with
    load_state_dict(strict=True) (model.py:165-209),
  - same methods and return shapes: forward (211-253), mc_inference (256-328),
    mc_inference_serial (330-401).
What differs, by design:
  - the dropout masks come from the MI355X Philox stream (oracle/philox_oracle.c documents it)
    instead of torch's global RNG; `seed=None` draws the Philox key from torch's default CPU
    generator, so torch.manual_seed(...) still makes a run reproducible (infer.py:137-145);
  - mc_inference and mc_inference_serial give identical samples for the same seed (the
    reference's two methods consume its RNG in different orders);
  - the head runs only on a HIP device and only without autograd: training (net_utils.py
    train_gacc) is out of scope and raises instead of silently running elsewhere.
Extra entry: mc_inference_features(H, T, seed, ...) starts at the kernel boundary (features).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .resnet import Identity, build_backbone

__all__ = ["MultiHeadGatedAttentionMIL", "AuxiliaryLoss"]


class AuxiliaryLoss(nn.Module):
    """Attention-head separation regulariser (reference model.py:405-438; training only)."""

    def __init__(self, loss_type="pairwise", margin=1.0, scale=1.0):
        super().__init__()
        self.loss_type = loss_type
        self.margin = margin
        self.scale = scale

    def forward(self, pos_attention, neg_attention, is_positive):
        if self.loss_type == "pairwise":
            d = F.pairwise_distance(pos_attention, neg_attention, p=2)
            return torch.mean((self.margin - d).clamp(min=0)) if is_positive else torch.mean(d)
        if self.loss_type == "cosine":
            cs = F.cosine_similarity(pos_attention, neg_attention, dim=1)
            return torch.mean(cs) if is_positive else torch.mean(1 - cs)
        raise ValueError(f"Unknown loss type: {self.loss_type}")


def _walk(root, path):
    """root._modules[path[0]]._modules[path[1]]... (KeyError if a link is gone)."""
    m = root
    for k in path:
        m = m._modules[k]
    return m


def _draw_seed() -> int:
    # key for the Philox stream, taken from torch's default CPU generator
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


class MultiHeadGatedAttentionMIL(nn.Module):
    def __init__(self, num_classes=2, backbone="r18", pretrained=True, L=512, D=128,
                 feature_dropout=0.1, attention_dropout=0.1, shared_attention=True,
                 neptune_run=None):
        super().__init__()
        self.auxiliary_loss = AuxiliaryLoss(loss_type="pairwise", margin=1.0, scale=.5)
        self.fold_idx = None
        self.neptune_run = neptune_run if neptune_run else None
        self.L = L
        self.D = D
        self.num_classes = num_classes
        self.shared_attention = shared_attention
        # reference model.py:166-177: without `pretrained` the reference always builds r18
        self.feature_extractor = build_backbone(backbone if pretrained else "r18", pretrained)
        self.feature_extractor.fc = Identity()
        if shared_attention:
            self.attention_V = nn.Sequential(nn.Linear(L, D), nn.Tanh())
            self.attention_U = nn.Sequential(nn.Linear(L, D), nn.Sigmoid())
        else:
            self.attention_V = nn.ModuleList([nn.Sequential(nn.Linear(L, D), nn.Tanh())
                                              for _ in range(num_classes)])
            self.attention_U = nn.ModuleList([nn.Sequential(nn.Linear(L, D), nn.Sigmoid())
                                              for _ in range(num_classes)])
        self.attention_weights = nn.ModuleList([nn.Linear(D, 1) for _ in range(num_classes)])
        self.classifiers = nn.ModuleList([nn.Linear(L, 1, bias=False) for _ in range(num_classes)])
        self.feature_dropout = nn.Dropout(feature_dropout)
        self.attention_dropouts = nn.ModuleList([nn.Dropout(attention_dropout)
                                                 for _ in range(num_classes)])
        # GEMM operand precision of the kernel: float32 (reference numerics) or bfloat16
        self.compute_dtype = torch.float32
        self._head_cache = None

    # ------------------------------------------------------------------ parameters
    def _gate_linears(self):
        if self.shared_attention:
            return [self.attention_V[0]], [self.attention_U[0]]
        return [m[0] for m in self.attention_V], [m[0] for m in self.attention_U]

    def _head_slots(self):
        """(module, parameter name) of every head parameter, in kernel order."""
        lv, lu = self._gate_linears()
        slots = [(m, n) for m in lv + lu for n in ("weight", "bias")]
        slots += [(m, n) for m in self.attention_weights for n in ("weight", "bias")]
        slots += [(m, "weight") for m in self.classifiers]
        return slots

    def _head_params(self):
        """The head's parameters in kernel order. The list is cached (the per-bag caller of
        infer.py:187-191 would otherwise walk nn.Module attribute lookups on every call) and
        revalidated on every call by identity, with plain dict lookups: every module on the path
        from self to each parameter's owner, and the Parameter object in its owner's _parameters.
        So replacing a Linear inside a container, assigning a new Parameter, or
        load_state_dict(..., assign=True) all miss the cache; the cache holds the objects it
        compares against, so an id cannot be reused while it is alive."""
        hit = self.__dict__.get("_head_param_cache")
        if hit is not None and self.shared_attention == hit[0]:
            chains, slots, params = hit[1:]
            try:
                ok = all(_walk(self, path) is m for path, m in chains) and \
                    all(m._parameters.get(n) is p for (m, n), p in zip(slots, params))
            except KeyError:
                ok = False
            if ok:
                return params
        slots = self._head_slots()
        params = [m._parameters[n] for m, n in slots]
        names = {id(m): name for name, m in self.named_modules()}
        owners = {id(m): m for m, _ in slots}
        chains = [(tuple(names[i].split(".")), m) for i, m in owners.items()]
        self.__dict__["_head_param_cache"] = (self.shared_attention, chains, slots, params)
        return params

    def head_tensors(self, device) -> ops.HeadTensors:
        """The head parameters stacked for the kernel (cached until a parameter changes)."""
        params = self._head_params()
        key = (str(device), self.compute_dtype,
               tuple((p.data_ptr(), p._version) for p in params))
        if self._head_cache is not None and self._head_cache[0] == key:
            return self._head_cache[1], self._head_cache[2]
        lv, lu = self._gate_linears()
        with torch.no_grad():
            f32 = dict(device=device, dtype=torch.float32)
            head = ops.HeadTensors(
                Wv=torch.stack([m.weight for m in lv]).to(**f32).contiguous(),
                bv=torch.stack([m.bias for m in lv]).to(**f32).contiguous(),
                Wu=torch.stack([m.weight for m in lu]).to(**f32).contiguous(),
                bu=torch.stack([m.bias for m in lu]).to(**f32).contiguous(),
                wa=torch.cat([m.weight for m in self.attention_weights]).to(**f32).contiguous(),
                ba=torch.cat([m.bias for m in self.attention_weights]).to(**f32).contiguous(),
                wk=torch.cat([m.weight for m in self.classifiers]).to(**f32).contiguous())
            packed = ops.packed_weights(head, self.compute_dtype)
        self._head_cache = (key, head, packed)
        return head, packed

    def _dropout_ps(self):
        """Active dropout probabilities: a layer applies dropout iff it is in train mode."""
        pf = self.feature_dropout.p if self.feature_dropout.training else 0.0
        pas = {d.p if d.training else 0.0 for d in self.attention_dropouts}
        if len(pas) != 1:
            raise NotImplementedError("per-class attention dropout rates / modes must agree")
        return pf, pas.pop()

    def _check_device(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("the MI355X MCDO head runs on a HIP device only "
                               f"(got device={device}); there is no CPU path")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        return device

    def _offsets(self, n, bs, device):
        """CSR offsets of bs bags of n instances, made on the device once per shape (infer.py:187-191
        calls mc_inference once per bag: no per-call host->device copy or allocation)."""
        key = (str(device), n, bs)
        cache = self.__dict__.setdefault("_offs_cache", {})
        t = cache.get(key)
        if t is None:
            if len(cache) > 64:
                cache.clear()
            t = cache[key] = ops.uniform_offsets(n, bs, device) if n > 0 else \
                ops.bag_offsets_tensor([0] * bs, device)
        return t

    # ------------------------------------------------------------------ kernel boundary
    def extract_features(self, x):
        """x [bs, n, 3, h, w] -> H [bs, n, L] (reference model.py:275-277)."""
        bs, n = x.shape[:2]
        H = self.feature_extractor(x.view(-1, *x.shape[-3:]))
        return H.view(bs, n, -1)

    @torch.no_grad()
    def mc_inference_features(self, H, T=30, seed=None, *, p_feat=None, p_att=None,
                              return_stats=False, bag_id_base=0, t_base=0):
        """MCDO over extracted features: H [n, L] or [bs, n, L] -> (Y [T, bs, C], A [T, bs, C, n])
        plus, with return_stats, a dict of A_mean/A_var [bs, C, n] and P_mean [bs, C]."""
        if H.dim() == 2:
            H = H.unsqueeze(0)
        device = self._check_device(H.device)
        bs, n, L = H.shape
        if seed is None:
            seed = _draw_seed()
        pf = self.feature_dropout.p if p_feat is None else p_feat
        pa = self.attention_dropouts[0].p if p_att is None else p_att
        head, packed = self.head_tensors(device)
        Hc = H.reshape(bs * n, L).to(self.compute_dtype).contiguous()
        offs = self._offsets(n, bs, device)
        out = ops.mcdo_forward(Hc, offs, head, T, p_feat=pf, p_att=pa, seed=seed,
                               bag_id_base=bag_id_base, t_base=t_base, packed=packed,
                               return_attention=True, return_stats=return_stats)
        C = self.num_classes
        Y = out["Y"].permute(1, 0, 2)                                   # [T, bs, C]
        A = out["A"].view(bs, T, C, n).permute(1, 0, 2, 3)              # [T, bs, C, n]
        if not return_stats:
            return Y, A
        stats = {"A_mean": out["A_mean"].view(bs, C, n), "A_var": out["A_var"].view(bs, C, n),
                 "P_mean": out["P_mean"]}
        return Y, A, stats

    # ------------------------------------------------------------------ reference API
    def forward(self, x, targets=None):
        """reference model.py:211-253. Returns (Y [bs, C], A_all [bs, C, n], aux_loss | None).
        Dropout is applied by the layers that are in train mode (eval(): none)."""
        if torch.is_grad_enabled() and self.training and any(p.requires_grad
                                                            for p in self.parameters()):
            raise NotImplementedError("training is out of scope for the MI355X MCDO build; "
                                      "call forward() in eval mode or under torch.no_grad()")
        with torch.no_grad():
            H = self.extract_features(x)
            pf, pa = self._dropout_ps()
            Y, A = self.mc_inference_features(H, T=1, p_feat=pf, p_att=pa)
        Y, A = Y[0], A[0]
        aux = None
        if targets is not None:
            is_positive = targets.item() == 1
            aux = self.auxiliary_loss.scale * self.auxiliary_loss(A[:, 1, :], A[:, 0, :],
                                                                  is_positive)
        return Y, A, aux

    def _enable_mc_dropout(self, device):
        # reference model.py:263-271 (the dropout layers stay in train mode afterwards)
        self.eval()
        self.to(device)

        def enable_dropout(m):
            if isinstance(m, nn.Dropout):
                m.train()
        self.apply(enable_dropout)

    @torch.no_grad()
    def mc_inference(self, input_tensor, N=30, device="cuda", targets=None, *, seed=None,
                     return_losses=False):
        """reference model.py:256-328: (Y [N, bs, C], A [N, bs, C, n]) for N MC samples.
        return_losses=True returns the 3-tuple (Y, A, losses) the reference's callers unpack
        (infer.py:191, net_utils.py:126,205)."""
        device = self._check_device(device)
        self._enable_mc_dropout(device)
        x = input_tensor.to(device)
        H = self.extract_features(x)
        pf, pa = self._dropout_ps()
        Y, A = self.mc_inference_features(H, T=N, seed=seed, p_feat=pf, p_att=pa)
        if not return_losses:
            return Y, A
        losses = None
        if targets is not None:
            is_positive = targets.item() == 1
            s = self.auxiliary_loss.scale
            losses = [s * self.auxiliary_loss(A[i, :, 1, :], A[i, :, 0, :], is_positive)
                      for i in range(N)]
        return Y, A, losses

    @torch.no_grad()
    def mc_inference_serial(self, input_tensor, N=30, device="cuda", *, seed=None):
        """reference model.py:330-401: one kernel launch per sample (sample counter t_base=t);
        same values as mc_inference with the same seed."""
        device = self._check_device(device)
        self._enable_mc_dropout(device)
        x = input_tensor.to(device)
        H = self.extract_features(x)
        pf, pa = self._dropout_ps()
        if seed is None:
            seed = _draw_seed()
        Ys, As = [], []
        for t in range(N):
            Y, A = self.mc_inference_features(H, T=1, seed=seed, p_feat=pf, p_att=pa, t_base=t)
            Ys.append(Y[0])
            As.append(A[0])
        return torch.stack(Ys), torch.stack(As)
