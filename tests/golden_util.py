"""Helpers shared by the oracle and GPU parity tests: load a golden fixture (outputs of the
reference module, tests/golden/make_golden.py) and regenerate its inputs and masks."""
import glob
import os

import numpy as np

from oracle import mcdo_ref, philox
from mcgmil import synthetic

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = ("N", "T", "C", "L", "D", "shared", "p_f", "p_a", "h_seed", "w_seed", "mask_seed",
        "bag_ctr", "bf16")


def names(prefix=""):
    """MCDO head golden cases (the patcher_* fixtures belong to tests/test_patcher_oracle.py, the
    caller_stats_* ones to tests/test_caller_stats.py)."""
    return sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, prefix + "*.npz"))
                  if not os.path.basename(f).startswith(("patcher_", "caller_stats_")))


class Case:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"))
        self.z = {k: z[k] for k in z.files}
        m = {k: self.z[k].item() for k in META}
        self.__dict__.update(m)
        self.shared = bool(self.shared)
        self.bf16 = bool(self.bf16)
        self.forward = name.startswith("forward")
        self.serial = name.startswith("serial")

    def inputs(self):
        H = synthetic.bag_features(self.h_seed, self.N, self.L)
        sd = synthetic.head_state_dict(self.w_seed, L=self.L, D=self.D, C=self.C,
                                       shared=self.shared)
        if self.bf16:
            H = synthetic.bf16_round(H)
            sd = synthetic.round_state_dict_bf16(sd)
        return H, sd, synthetic.head_arrays(sd, self.C, self.shared)

    def masks(self):
        return mcdo_ref.masks_for_bag(self.mask_seed, self.bag_ctr, self.T, self.N, self.L,
                                      self.C, self.p_f, self.p_a)

    def feature_bits(self):
        return philox.feature_keep_bits(self.mask_seed, self.bag_ctr, self.T, self.N, self.L,
                                        self.p_f)


def nrel(got, ref):
    """max|got - ref| / max|ref|."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if not ref.size:
        return 0.0
    den = np.max(np.abs(ref))
    return float(np.max(np.abs(got - ref)) / (den if den > 0 else 1.0))
