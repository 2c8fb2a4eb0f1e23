"""TEST INFRASTRUCTURE -- the statistics the reference's callers derive from mc_inference's
(Y, A), restated in numpy. Only tests/ import this, as the checker of mcgmil.infer.

Reference lines restated (xkuubix/MonteCarlo-Gated-MIL):
  infer.py:195        probs = softmax(ys, dim=-1)                      (over classes, per pass)
  infer.py:18-19      neg/pos attention scaling factors = probs[:, :, c].mean()
  infer.py:47-54      positive-class probabilities over the passes: np.mean, np.median,
                      np.std (ddof=0), np.percentile(75) - np.percentile(25), np.min, np.max
  infer.py:56-57      entropy = -sum_c p log(p + 1e-10) per pass, then its mean
  net_utils.py:207-210  mc_test: softmax -> mean over passes -> argmax
  infer.py:216-219    attention mean and torch's unbiased std over passes (var = std^2)

Parity: pinned. The reference's own plot_attention_and_density (infer.py:14-92) was run on the
reference's MC logits (and seeded random ones) by tests/golden/make_golden_stats.py, which
compiles only that function from /root/reference/infer.py (the module itself imports neptune,
matplotlib and the DICOM dataset, absent here) and captures its mean/median/std/IQR/min/max and
mean entropy from a recording matplotlib stand-in; tests/golden/caller_stats_ref.npz holds them
and tests/test_caller_stats.py checks this restatement against them (|diff| <= 1e-6).
"""
import numpy as np


def softmax_classes(Y):
    """infer.py:195 -- Y [T, C] (raw logits, one row per pass) -> probabilities, float32."""
    Y = np.asarray(Y, dtype=np.float32)
    e = np.exp(Y - Y.max(axis=-1, keepdims=True))
    return (e / e.sum(axis=-1, keepdims=True)).astype(np.float32)


def caller_stats(Y, A=None):
    """Everything infer.py / net_utils.py compute per bag from Y [T, C] (and A [T, C, N])."""
    probs = softmax_classes(Y)                       # [T, C]
    pos = probs[:, -1]                               # infer.py:47 positive class (C = 2: index 1)
    out = {
        "probs": probs,
        "prob_mean": probs.mean(axis=0),                                   # net_utils.py:208
        "prediction": int(np.argmax(probs.mean(axis=0))),                  # net_utils.py:210
        "scaling": probs.mean(axis=0),                                     # infer.py:18-19
        "pos_mean": float(np.mean(pos)),                                   # infer.py:49
        "pos_median": float(np.median(pos)),                               # infer.py:50
        "pos_std": float(np.std(pos)),                                     # infer.py:51 (ddof=0)
        "pos_iqr": float(np.percentile(pos, 75) - np.percentile(pos, 25)),  # infer.py:52
        "pos_min": float(np.min(pos)), "pos_max": float(np.max(pos)),       # infer.py:53
    }
    ent = -np.sum(probs * np.log(probs + np.float32(1e-10)), axis=-1)      # infer.py:56
    out["mean_entropy"] = float(ent.mean())                                # infer.py:57
    if A is not None:
        A = np.asarray(A, dtype=np.float64)
        T = A.shape[0]
        out["A_mean"] = A.mean(axis=0)                                     # infer.py:216
        out["A_var"] = A.var(axis=0, ddof=1) if T > 1 else np.full(A.shape[1:], np.nan)  # 217-219
    return out
