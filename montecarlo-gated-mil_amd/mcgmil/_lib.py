"""ctypes binding of the C ABI in include/mcgmil.h (libmcgmil.so, built for gfx950).

torch is imported first on purpose: torch ships the HIP runtime (SONAME libamdhip64.so.7), and
the library's NEEDED entry then resolves to that already-loaded copy, so the kernels run on
torch's device context and streams.

There is no fallback: if the library is missing or fails to load, every call raises.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before the library)

from . import _build

MCGMIL_F32 = 0
MCGMIL_BF16 = 1
MCGMIL_U8 = 2
MCGMIL_U16 = 3

ABI_VERSION = 6
# mcgmil_args.flags (include/mcgmil.h enum mcgmil_flags)
PATH_FLAGS = {"auto": 0, "fused": 1, "two_kernel": 2}
# mcgmil_conv_args.flags / mcgmil_stem_args.flags (include/mcgmil_features.h)
CONV_TILE_FLAGS = {"auto": 0, "nohalo": 1, "small": 2, "big512": 3}
STEM_POOL_UNSPLIT = 1
GATE_FLAGS = {"auto": 0, "pipe": 1 << 2, "pp": 2 << 2}
CLOCK_PROBE = 1 << 4         # MCGMIL_CLOCK_PROBE: clock record of the gate launch into args.debug
CLOCK_SLOTS = 1024           # MCGMIL_CLOCK_SLOTS: [slots][4] uint64

EXPORTED = (
    "mcgmil_abi_version", "mcgmil_args_size", "mcgmil_last_error", "mcgmil_workspace_size",
    "mcgmil_packed_weights_size", "mcgmil_pack_weights", "mcgmil_mcdo_forward",
    "mcgmil_gate_softmax_pool", "mcgmil_fused_regions", "mcgmil_gate_scores", "mcgmil_softmax_pool", "mcgmil_bag_stats", "mcgmil_feature_keep",
    "mcgmil_attention_keep",
    # include/mcgmil_image.h
    "mcgmil_image_args_size", "mcgmil_tile_grid", "mcgmil_image_workspace_size",
    "mcgmil_image_to_bag", "mcgmil_attention_maps", "mcgmil_reconstruct_image",
    # include/mcgmil_features.h
    "mcgmil_bn_args_size", "mcgmil_bn_workspace_size", "mcgmil_batchnorm_act",
    "mcgmil_batchnorm_coefficients", "mcgmil_conv_input_bn",
    "mcgmil_conv_args_size", "mcgmil_pack_conv_weights", "mcgmil_conv_stats_parts", "mcgmil_conv2d",
    "mcgmil_conv_workspace_size",
    "mcgmil_conv_packed_size_f32", "mcgmil_pack_conv_weights_f32", "mcgmil_conv2d_f32",
    "mcgmil_conv_stats_parts_f32",
    "mcgmil_stem_args_size", "mcgmil_stem_packed_size", "mcgmil_pack_stem_weights",
    "mcgmil_stem_workspace_size", "mcgmil_stem_forward",
    # include/mcgmil_calib.h (measurement)
    "mcgmil_mfma_calib_flops_per_step", "mcgmil_mfma_calib",
)

_vp = ctypes.c_void_p


class Args(ctypes.Structure):
    """Mirror of struct mcgmil_args (include/mcgmil.h); field order and types must match."""
    _fields_ = [
        ("L", ctypes.c_int32), ("D", ctypes.c_int32), ("C", ctypes.c_int32),
        ("G", ctypes.c_int32), ("T", ctypes.c_int32), ("num_bags", ctypes.c_int32),
        ("total_rows", ctypes.c_int64),
        ("h_dtype", ctypes.c_int32), ("uniform_bag_rows", ctypes.c_int32),
        ("H", _vp), ("ldh", ctypes.c_int64), ("bag_offsets", _vp),
        ("Wv", _vp), ("bv", _vp), ("Wu", _vp), ("bu", _vp), ("wa", _vp), ("ba", _vp),
        ("wk", _vp), ("packed_w", _vp),
        ("p_feat", ctypes.c_float), ("p_att", ctypes.c_float), ("seed", ctypes.c_uint64),
        ("bag_id_base", ctypes.c_uint32), ("t_base", ctypes.c_int32), ("bag_ids", _vp),
        ("keep_feat", _vp), ("keep_att", _vp),
        ("Y", _vp), ("A", _vp), ("A_mean", _vp), ("A_var", _vp), ("P_mean", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t), ("debug", _vp),
        ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class ImageArgs(ctypes.Structure):
    """Mirror of struct mcgmil_image_args (include/mcgmil_image.h)."""
    _fields_ = [
        ("height", ctypes.c_int32), ("width", ctypes.c_int32), ("channels", ctypes.c_int32),
        ("patch_size", ctypes.c_int32), ("overlap", ctypes.c_double),
        ("empty_thresh", ctypes.c_double), ("bag_size", ctypes.c_int32),
        ("shuffle", ctypes.c_int32), ("shuffle_seed", ctypes.c_uint64),
        ("image_dtype", ctypes.c_int32), ("out_dtype", ctypes.c_int32),
        ("normalize", ctypes.c_int32), ("norm_mean", ctypes.c_float * 4),
        ("norm_std", ctypes.c_float * 4), ("image", _vp),
        ("ld_row", ctypes.c_int64), ("ld_channel", ctypes.c_int64),
        ("px", _vp), ("tile_ids", _vp), ("num_selected", _vp), ("instances", _vp),
        ("instance_capacity", ctypes.c_int32),
        ("T", ctypes.c_int32), ("C", ctypes.c_int32), ("k", ctypes.c_int32),
        ("attention", _vp), ("map_tile_ids", _vp), ("maps", _vp), ("map_mean", _vp),
        ("map_std", _vp), ("patches", _vp), ("image_out", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class ConvArgs(ctypes.Structure):
    """Mirror of struct mcgmil_conv_args (include/mcgmil_features.h)."""
    _fields_ = [
        ("batch", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
        ("in_channels", ctypes.c_int32), ("out_channels", ctypes.c_int32),
        ("kernel_h", ctypes.c_int32), ("kernel_w", ctypes.c_int32), ("stride", ctypes.c_int32),
        ("pad", ctypes.c_int32), ("in_relu", ctypes.c_int32),
        ("x", _vp), ("w", _vp), ("y", _vp), ("stats", _vp), ("in_ab", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
        ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class StemArgs(ctypes.Structure):
    """Mirror of struct mcgmil_stem_args (include/mcgmil_features.h)."""
    _fields_ = [
        ("batch", ctypes.c_int32), ("in_channels", ctypes.c_int32), ("height", ctypes.c_int32),
        ("width", ctypes.c_int32), ("out_channels", ctypes.c_int32), ("kernel", ctypes.c_int32),
        ("stride", ctypes.c_int32), ("pad", ctypes.c_int32), ("pool_kernel", ctypes.c_int32),
        ("pool_stride", ctypes.c_int32), ("pool_pad", ctypes.c_int32), ("relu", ctypes.c_int32),
        ("eps", ctypes.c_double), ("x", _vp), ("w", _vp), ("gamma", _vp), ("beta", _vp),
        ("running_mean", _vp), ("running_var", _vp), ("y", _vp),
        ("batch_mean", _vp), ("batch_invstd", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
        ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class BnArgs(ctypes.Structure):
    """Mirror of struct mcgmil_bn_args (include/mcgmil_features.h)."""
    _fields_ = [
        ("rows", ctypes.c_int64), ("channels", ctypes.c_int32), ("dtype", ctypes.c_int32),
        ("x", _vp), ("residual", _vp), ("y", _vp), ("gamma", _vp), ("beta", _vp),
        ("running_mean", _vp), ("running_var", _vp), ("eps", ctypes.c_double),
        ("relu", ctypes.c_int32), ("batch", ctypes.c_int32), ("height", ctypes.c_int32),
        ("width", ctypes.c_int32), ("pool_kernel", ctypes.c_int32), ("pool_stride", ctypes.c_int32),
        ("pool_pad", ctypes.c_int32), ("num_partials", ctypes.c_int32),
        ("batch_mean", _vp), ("batch_invstd", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t), ("partials", _vp),
        ("residual_ab", _vp),
    ]


class MCGMILError(RuntimeError):
    pass


_lib = None


def lib_path() -> str:
    # MCGMIL_LIB: an A/B build of the same library (timing studies); default the in-tree build
    return os.environ.get("MCGMIL_LIB", _build.LIB)


def load():
    """Load libmcgmil.so (raises if it was not built -- there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise MCGMILError(f"MI355X extension not built: {path} is missing "
                          "(run __graft_entry__.build() or python -m mcgmil._build)")
    _lib = bind(path)
    return _lib


def bind(path: str, mcdo_only: bool = False, any_abi: bool = False):
    """dlopen a build of the library and declare its entry points. mcdo_only: a gate-kernel A/B
    build (scripts/build_variants.sh with GATE_ONLY=1) that holds the MCDO entry points only;
    any_abi: an A/B build of an earlier revision (same mcgmil_args layout, older ABI number)."""
    L = ctypes.CDLL(path)
    pa = ctypes.POINTER(Args)
    L.mcgmil_abi_version.restype = ctypes.c_int
    L.mcgmil_args_size.restype = ctypes.c_size_t
    L.mcgmil_last_error.restype = ctypes.c_char_p
    for name in ("mcgmil_workspace_size", "mcgmil_packed_weights_size"):
        f = getattr(L, name)
        f.argtypes = [pa, ctypes.POINTER(ctypes.c_size_t)]
        f.restype = ctypes.c_int
    L.mcgmil_pack_weights.argtypes = [pa, _vp, _vp]
    L.mcgmil_pack_weights.restype = ctypes.c_int
    for name in ("mcgmil_mcdo_forward", "mcgmil_gate_softmax_pool", "mcgmil_gate_scores",
                 "mcgmil_softmax_pool", "mcgmil_bag_stats"):
        f = getattr(L, name)
        f.argtypes = [pa, _vp]
        f.restype = ctypes.c_int
    L.mcgmil_fused_regions.argtypes = [pa, ctypes.POINTER(ctypes.c_int64)]
    L.mcgmil_fused_regions.restype = ctypes.c_int
    for name in ("mcgmil_feature_keep", "mcgmil_attention_keep"):
        f = getattr(L, name)
        f.argtypes = [pa, _vp, _vp]
        f.restype = ctypes.c_int
    if L.mcgmil_abi_version() != ABI_VERSION and not any_abi:
        raise MCGMILError(f"ABI mismatch: {path} has ABI version {L.mcgmil_abi_version()}, "
                          f"the binding expects {ABI_VERSION}")
    if L.mcgmil_args_size() != ctypes.sizeof(Args):
        raise MCGMILError(f"ABI mismatch: sizeof(mcgmil_args)={L.mcgmil_args_size()} but the "
                          f"ctypes mirror is {ctypes.sizeof(Args)} bytes")
    if mcdo_only:
        return L
    pi = ctypes.POINTER(ImageArgs)
    L.mcgmil_image_args_size.restype = ctypes.c_size_t
    L.mcgmil_tile_grid.argtypes = [pi, _vp, _vp, _vp, _vp]
    L.mcgmil_tile_grid.restype = ctypes.c_int
    L.mcgmil_image_workspace_size.argtypes = [pi, ctypes.POINTER(ctypes.c_size_t)]
    L.mcgmil_image_workspace_size.restype = ctypes.c_int
    for name in ("mcgmil_image_to_bag", "mcgmil_attention_maps", "mcgmil_reconstruct_image"):
        f = getattr(L, name)
        f.argtypes = [pi, _vp]
        f.restype = ctypes.c_int
    pb = ctypes.POINTER(BnArgs)
    L.mcgmil_bn_args_size.restype = ctypes.c_size_t
    L.mcgmil_bn_workspace_size.argtypes = [pb, ctypes.POINTER(ctypes.c_size_t)]
    L.mcgmil_bn_workspace_size.restype = ctypes.c_int
    L.mcgmil_batchnorm_act.argtypes = [pb, _vp]
    L.mcgmil_batchnorm_act.restype = ctypes.c_int
    L.mcgmil_batchnorm_coefficients.argtypes = [pb, _vp, _vp]
    L.mcgmil_batchnorm_coefficients.restype = ctypes.c_int
    pc = ctypes.POINTER(ConvArgs)
    L.mcgmil_conv_args_size.restype = ctypes.c_size_t
    L.mcgmil_pack_conv_weights.argtypes = [pc, _vp, ctypes.c_int32, _vp, _vp]
    L.mcgmil_pack_conv_weights.restype = ctypes.c_int
    L.mcgmil_conv_stats_parts.argtypes = [pc, ctypes.POINTER(ctypes.c_int32)]
    L.mcgmil_conv_stats_parts.restype = ctypes.c_int
    L.mcgmil_conv_input_bn.argtypes = [pc, ctypes.POINTER(ctypes.c_int32)]
    L.mcgmil_conv_input_bn.restype = ctypes.c_int
    L.mcgmil_conv2d.argtypes = [pc, _vp]
    L.mcgmil_conv2d.restype = ctypes.c_int
    L.mcgmil_conv_workspace_size.argtypes = [pc, ctypes.POINTER(ctypes.c_size_t)]
    L.mcgmil_conv_workspace_size.restype = ctypes.c_int
    L.mcgmil_conv_packed_size_f32.argtypes = [pc, ctypes.POINTER(ctypes.c_size_t)]
    L.mcgmil_conv_packed_size_f32.restype = ctypes.c_int
    L.mcgmil_conv_stats_parts_f32.argtypes = [pc, ctypes.POINTER(ctypes.c_int32)]
    L.mcgmil_conv_stats_parts_f32.restype = ctypes.c_int
    L.mcgmil_pack_conv_weights_f32.argtypes = [pc, _vp, _vp, _vp]
    L.mcgmil_pack_conv_weights_f32.restype = ctypes.c_int
    L.mcgmil_conv2d_f32.argtypes = [pc, _vp]
    L.mcgmil_conv2d_f32.restype = ctypes.c_int
    ps = ctypes.POINTER(StemArgs)
    L.mcgmil_stem_args_size.restype = ctypes.c_size_t
    for name in ("mcgmil_stem_packed_size", "mcgmil_stem_workspace_size"):
        f = getattr(L, name)
        f.argtypes = [ps, ctypes.POINTER(ctypes.c_size_t)]
        f.restype = ctypes.c_int
    L.mcgmil_pack_stem_weights.argtypes = [ps, _vp, ctypes.c_int32, _vp, _vp]
    L.mcgmil_pack_stem_weights.restype = ctypes.c_int
    L.mcgmil_stem_forward.argtypes = [ps, _vp]
    L.mcgmil_stem_forward.restype = ctypes.c_int
    L.mcgmil_mfma_calib_flops_per_step.argtypes = [ctypes.c_int]
    L.mcgmil_mfma_calib_flops_per_step.restype = ctypes.c_int64
    L.mcgmil_mfma_calib.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _vp, _vp, _vp]
    L.mcgmil_mfma_calib.restype = ctypes.c_int
    if L.mcgmil_stem_args_size() != ctypes.sizeof(StemArgs):
        raise MCGMILError(f"ABI mismatch: sizeof(mcgmil_stem_args)={L.mcgmil_stem_args_size()} "
                          f"but the ctypes mirror is {ctypes.sizeof(StemArgs)} bytes")
    if L.mcgmil_conv_args_size() != ctypes.sizeof(ConvArgs):
        raise MCGMILError(f"ABI mismatch: sizeof(mcgmil_conv_args)={L.mcgmil_conv_args_size()} "
                          f"but the ctypes mirror is {ctypes.sizeof(ConvArgs)} bytes")
    if L.mcgmil_bn_args_size() != ctypes.sizeof(BnArgs):
        raise MCGMILError(f"ABI mismatch: sizeof(mcgmil_bn_args)={L.mcgmil_bn_args_size()} "
                          f"but the ctypes mirror is {ctypes.sizeof(BnArgs)} bytes")
    if L.mcgmil_image_args_size() != ctypes.sizeof(ImageArgs):
        raise MCGMILError(f"ABI mismatch: sizeof(mcgmil_image_args)={L.mcgmil_image_args_size()} "
                          f"but the ctypes mirror is {ctypes.sizeof(ImageArgs)} bytes")
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = load().mcgmil_last_error().decode(errors="replace")
        raise MCGMILError(f"{what} failed ({rc}): {msg}")
