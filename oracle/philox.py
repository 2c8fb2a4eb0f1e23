"""TEST INFRASTRUCTURE -- Python binding of the C mask oracle (oracle/philox_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
The mask stream it defines replaces torch's CPU RNG used by the reference's dropout layers
(reference model.py:280-281 feature dropout, model.py:291/301 attention dropout); see the
header of philox_oracle.c for the exact rule.
"""
import ctypes

import numpy as np

from . import build as _build

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = _build.build()
        L = ctypes.CDLL(path)
        L.oracle_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_philox4x32_10.restype = None
        L.oracle_drop_threshold.argtypes = [ctypes.c_double]
        L.oracle_drop_threshold.restype = ctypes.c_uint32
        L.oracle_dropout_scale.argtypes = [ctypes.c_double]
        L.oracle_dropout_scale.restype = ctypes.c_float
        L.oracle_feature_keep.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_feature_keep.restype = ctypes.c_int
        L.oracle_attention_keep.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_attention_keep.restype = ctypes.c_int
        _lib = L
    return _lib


def philox4x32_10(ctr, key):
    c = (ctypes.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (ctypes.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return [int(x) for x in o]


def philox4x32_10_py(ctr, key):
    """Independent pure-Python restatement, used only to cross-check the C one."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c0, c1, c2, c3 = [int(x) & 0xFFFFFFFF for x in ctr]
    k0, k1 = [int(x) & 0xFFFFFFFF for x in key]
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, \
                         ((p0 >> 32) ^ c3 ^ k1) & 0xFFFFFFFF, p0 & 0xFFFFFFFF
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [c0, c1, c2, c3]


def drop_threshold(p: float) -> int:
    return int(lib().oracle_drop_threshold(float(p)))


def dropout_scale(p: float) -> float:
    return float(lib().oracle_dropout_scale(float(p)))


def feature_keep_bits(seed, bag_ctr, T, N, L, p, t0=0):
    """Packed keep bits [T, N, L//8] uint8 (bit l&7 of byte l>>3)."""
    out = np.empty((T, N, L // 8), dtype=np.uint8)
    rc = lib().oracle_feature_keep(int(seed) & (2**64 - 1), int(bag_ctr) & 0xFFFFFFFF, int(t0),
                                   int(T), int(N), int(L), drop_threshold(p),
                                   out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise ValueError("oracle_feature_keep rejected the shape")
    return out


def unpack_feature_bits(bits, L):
    """[T, N, L//8] packed -> [T, N, L] bool."""
    return np.unpackbits(bits, axis=-1, bitorder="little")[..., :L].astype(bool)


def pack_feature_bits(keep):
    """[T, N, L] bool -> [T, N, L//8] packed uint8."""
    return np.packbits(keep.astype(np.uint8), axis=-1, bitorder="little")


def feature_keep(seed, bag_ctr, T, N, L, p, t0=0):
    return unpack_feature_bits(feature_keep_bits(seed, bag_ctr, T, N, L, p, t0), L)


def attention_keep(seed, bag_ctr, T, C, N, p, t0=0):
    """Keep flags [T, C, N] bool."""
    out = np.empty((T, C, N), dtype=np.uint8)
    rc = lib().oracle_attention_keep(int(seed) & (2**64 - 1), int(bag_ctr) & 0xFFFFFFFF, int(t0),
                                     int(T), int(C), int(N), drop_threshold(p),
                                     out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise ValueError("oracle_attention_keep rejected the shape")
    return out.astype(bool)
