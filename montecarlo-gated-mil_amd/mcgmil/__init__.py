"""mcgmil -- MI355X-native Monte-Carlo-dropout gated-attention MIL inference.

Drop-in for the hot path of xkuubix/MonteCarlo-Gated-MIL (MultiHeadGatedAttentionMIL in the
reference model.py): the MCDO x gated-attention x classifier block runs as hand-written gfx950
HIP kernels behind the C ABI in include/mcgmil.h (libmcgmil.so, loaded with ctypes).

  model.MultiHeadGatedAttentionMIL   the reference nn.Module API (ctor, state_dict, forward,
                                     mc_inference, mc_inference_serial) + mc_inference_features
  ops.mcdo_forward                   batched varlen entry (many bags x T samples, one launch)
  library                            torch.ops.mcgmil.mcdo_forward(_stats): the same entry as
                                     torch.library custom ops (fake kernels for graph capture)
  infer.mc_predict_bags              caller-side uncertainty summary (reference infer.py)
  shard                              bag sharding + prediction gather across GPUs
  resnet                             in-repo ResNet backbone (torchvision is not available)
  patcher.ImagePatcher               the reference ImagePatcher on the GPU (tiling, selection,
                                     gather, attention maps + mean/std), include/mcgmil_image.h
"""
from .model import MultiHeadGatedAttentionMIL, AuxiliaryLoss  # noqa: F401
from .resnet import deactivate_batchnorm, Identity  # noqa: F401

__version__ = "0.1.0"
