"""Pin the caller-side uncertainty scalars (reference infer.py:47-57) with the REFERENCE's own code.

The reference computes them inside `plot_attention_and_density` (infer.py:14-92), which only
draws them into a matplotlib figure and returns nothing; infer.py itself cannot be imported here
(it imports neptune, matplotlib and the DICOM dataset module at module level). So this script
parses /root/reference/infer.py, compiles ONLY that function's definition with numpy and torch,
and gives it a recording stand-in for `plt`: the stand-in's `fig.text(...)` (infer.py:78) reads
the calling frame's locals, i.e. the reference's own mean_pred / median_pred / std_pred /
iqr_pred / min_pred / max_pred / mean_entropy, at full precision.

Inputs: the reference's own MC logits from the model fixtures (tests/golden/*.npz, Y [T, 1, C]),
turned into probabilities exactly as infer.py:195 does (softmax over the last dim), plus a few
seeded random logit sets. Output: tests/golden/caller_stats_ref.npz (inputs + the captured
scalars). Runs only where the read-only reference checkout exists; never on the GPU box.

Usage:  python tests/golden/make_golden_stats.py
"""
import ast
import os
import sys

import numpy as np
import torch

REF = "/root/reference/infer.py"
OUT = os.path.dirname(os.path.abspath(__file__))
FIXTURES = ("cfg2_N512_T30_sep", "cfg3_N2048_T100_sep", "small_N64_T4_shared", "edge_N100_T7_sep_p05",
            "serial_N64_T4_sep", "big_N5500_T4_sep")
CAPTURE = ("mean_pred", "median_pred", "std_pred", "iqr_pred", "min_pred", "max_pred", "mean_entropy")


class _Recorder:
    """Stand-in for matplotlib.pyplot and its figure/axes: every call is a no-op except
    Figure.text, which records the reference function's locals named in CAPTURE."""

    def __init__(self):
        self.captured = None

    def __getattr__(self, name):
        return self._noop

    def _noop(self, *a, **k):
        return self

    def __getitem__(self, key):
        return self

    def figure(self, *a, **k):
        return self

    def text(self, *a, **k):
        loc = sys._getframe(1).f_locals
        self.captured = {n: float(loc[n]) for n in CAPTURE}
        return self


def reference_function(rec):
    src = open(REF).read()
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "plot_attention_and_density")
    mod = ast.Module(body=[fn], type_ignores=[])
    ns = {"np": np, "torch": torch, "plt": rec}
    exec(compile(mod, REF, "exec"), ns)
    return ns["plot_attention_and_density"]


def main():
    rec = _Recorder()
    fn = reference_function(rec)
    logits, names, stats = [], [], []
    sets = []
    for name in FIXTURES:
        Y = np.load(os.path.join(OUT, name + ".npz"))["Y"]            # [T, 1, C] as mc_inference returns
        sets.append((name, Y.astype(np.float32)))
    rng = np.random.default_rng(7)
    for T in (2, 3, 50, 100):
        sets.append((f"random_T{T}", (rng.standard_normal((T, 1, 2)) * 3).astype(np.float32)))
    for name, Y in sets:
        assert Y.shape[0] > 1 and Y.shape[-1] == 2, (name, Y.shape)   # squeeze() needs T > 1; pos = class 1
        probs = torch.nn.functional.softmax(torch.from_numpy(Y), dim=-1)   # infer.py:195
        z = np.zeros((4, 4), np.float32)
        rec.captured = None
        fn(torch.zeros(3, 4, 4), z, z, z, z, probs, {"target": {"class": ["x"]}}, save_path=None)
        assert rec.captured is not None, name
        names.append(name)
        logits.append(Y[:, 0, :])
        stats.append([rec.captured[n] for n in CAPTURE])
        print(name, {k: round(v, 6) for k, v in rec.captured.items()})
    T_max = max(y.shape[0] for y in logits)
    padded = np.full((len(logits), T_max, 2), np.nan, np.float32)
    for i, y in enumerate(logits):
        padded[i, :y.shape[0]] = y
    np.savez(os.path.join(OUT, "caller_stats_ref.npz"), names=np.array(names), Y=padded,
             T=np.array([y.shape[0] for y in logits]), stats=np.array(stats, np.float64),
             keys=np.array(CAPTURE))
    print("wrote caller_stats_ref.npz")


if __name__ == "__main__":
    main()
