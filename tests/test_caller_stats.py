"""Caller-side uncertainty statistics (reference infer.py:47-57, 195; net_utils.py:205-210):
mcgmil.infer against the numpy restatement oracle/caller_stats.py, on the reference's own
logits (golden fixtures) and on random logits."""
import numpy as np
import pytest
import torch

from golden_util import Case
from oracle import caller_stats

KEYS = ("pos_mean", "pos_median", "pos_std", "pos_iqr", "pos_min", "pos_max", "mean_entropy")


def _check(got, want):
    np.testing.assert_allclose(got["probs"].cpu().numpy(), want["probs"], rtol=0, atol=3e-7)   # 2 ulp of 1.0
    np.testing.assert_allclose(got["prob_mean"].cpu().numpy(), want["prob_mean"], atol=3e-7)
    assert got["prediction"] == want["prediction"]
    for k in KEYS:
        assert abs(got[k] - want[k]) <= 1e-6, (k, got[k], want[k])


@pytest.mark.parametrize("name", ["cfg2_N512_T30_sep", "cfg3_N2048_T100_sep", "small_N64_T4_shared",
                                  "edge_N100_T7_sep_p05"])
def test_summary_of_reference_logits(name):
    """The reference's own Y (golden fixture) summarised both ways."""
    from mcgmil.infer import uncertainty_summary
    case = Case(name)
    Y = case.z["Y"][:, 0]                                   # [T, C]
    _check(uncertainty_summary(torch.from_numpy(Y)), caller_stats.caller_stats(Y))
    # the golden P_mean is the reference's softmax -> mean over passes (net_utils.py:207-208)
    np.testing.assert_allclose(caller_stats.caller_stats(Y)["prob_mean"], case.z["P_mean"], atol=1e-6)


@pytest.mark.parametrize("T", [1, 2, 3, 50, 100])
def test_summary_random_logits(T):
    from mcgmil.infer import uncertainty_summary
    rng = np.random.default_rng(T)
    Y = (rng.standard_normal((T, 2)) * 3).astype(np.float32)
    _check(uncertainty_summary(torch.from_numpy(Y)), caller_stats.caller_stats(Y))


def test_oracle_matches_numpy_definitions():
    """Spot-check the restatement itself: percentile IQR, ddof=0 std, entropy with +1e-10."""
    Y = np.array([[0.0, 1.0], [2.0, -1.0], [0.5, 0.5], [-3.0, 3.0]], np.float32)
    s = caller_stats.caller_stats(Y)
    p = np.exp(Y) / np.exp(Y).sum(-1, keepdims=True)
    pos = p[:, 1]
    assert abs(s["pos_iqr"] - (np.quantile(pos, 0.75) - np.quantile(pos, 0.25))) < 1e-6
    assert abs(s["pos_std"] - np.sqrt(np.mean((pos - pos.mean()) ** 2))) < 1e-6
    assert abs(s["mean_entropy"] - np.mean(-np.sum(p * np.log(p + 1e-10), -1))) < 1e-6
    assert s["prediction"] == int(np.argmax(p.mean(0)))


def _reference_stats():
    """tests/golden/caller_stats_ref.npz: the scalars the reference's own plot_attention_and_density
    computed (infer.py:47-57, captured by tests/golden/make_golden_stats.py) on the reference's
    MC logits and on seeded random logits."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "caller_stats_ref.npz"))
    keys = [str(k) for k in z["keys"]]
    for i, name in enumerate(z["names"]):
        T = int(z["T"][i])
        yield str(name), z["Y"][i, :T], dict(zip(keys, z["stats"][i].tolist()))


# reference local name (infer.py:49-57) -> caller_stats / uncertainty_summary key
REF_KEYS = {"mean_pred": "pos_mean", "median_pred": "pos_median", "std_pred": "pos_std",
            "iqr_pred": "pos_iqr", "min_pred": "pos_min", "max_pred": "pos_max",
            "mean_entropy": "mean_entropy"}


def test_oracle_matches_reference_scalars():
    """The restatement against the reference's own numbers (pinned, not restated)."""
    n = 0
    for name, Y, ref in _reference_stats():
        got = caller_stats.caller_stats(Y)
        for rk, k in REF_KEYS.items():
            assert abs(got[k] - ref[rk]) <= 1e-6, (name, k, got[k], ref[rk])
        n += 1
    assert n == 10


def _summary_matches_reference(device):
    from mcgmil.infer import uncertainty_summary
    for name, Y, ref in _reference_stats():
        got = uncertainty_summary(torch.from_numpy(Y).to(device))
        for rk, k in REF_KEYS.items():
            assert abs(got[k] - ref[rk]) <= 1e-6, (name, k, got[k], ref[rk])


def test_summary_matches_reference_scalars_cpu():
    _summary_matches_reference("cpu")


@pytest.mark.gpu
def test_summary_matches_reference_scalars_gpu():
    _summary_matches_reference("cuda")
