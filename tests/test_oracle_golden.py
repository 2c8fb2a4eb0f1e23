"""The CPU oracle (oracle/mcdo_ref.py) against the reference module's own outputs
(tests/golden/*.npz, produced by tests/golden/make_golden.py from /root/reference model.py with
replayed masks). This pins the oracle before it is used to check the HIP kernels."""
import numpy as np
import pytest
import torch

from oracle import mcdo_ref
from golden_util import Case, names, nrel

ALL = names()


def test_fixtures_present():
    assert len(ALL) >= 20, ALL


@pytest.mark.parametrize("name", ALL)
def test_oracle_matches_reference(name):
    case = Case(name)
    H, _, arrays = case.inputs()
    prm = mcdo_ref.HeadParams(arrays)
    if case.forward:
        Y, A = mcdo_ref.forward_eval(H, prm)
        np.testing.assert_allclose(Y.numpy(), case.z["Y"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(A.numpy(), case.z["A"], rtol=0, atol=1e-7)
        return
    kF, kA = case.masks()
    Y, A = mcdo_ref.mc_inference(H, prm, kF, kA, case.p_f, case.p_a)
    # same torch CPU op sequence -> agreement to fp32 rounding (bit-exact on this container)
    tol_y = 1e-5 if case.serial else 1e-6   # serial: reference loops per sample (other op order)
    np.testing.assert_allclose(Y.numpy(), case.z["Y"], rtol=0, atol=tol_y)
    if "A" in case.z:
        assert nrel(A.numpy(), case.z["A"]) <= 1e-6
    else:
        assert nrel(A[0].numpy(), case.z["A_first"]) <= 1e-6
        assert nrel(A[-1].numpy(), case.z["A_last"]) <= 1e-6
    Am, Av, Pm = mcdo_ref.uncertainty_stats(Y, A)
    assert nrel(Am.numpy(), case.z["A_mean"]) <= 1e-6
    if case.T > 1:
        assert nrel(Av.numpy(), case.z["A_var"]) <= 1e-5
    else:
        assert np.isnan(case.z["A_var"]).all() and torch.isnan(Av).all()
    np.testing.assert_allclose(Pm.numpy(), case.z["P_mean"], rtol=0, atol=1e-6)


def test_p0_mc_inference_equals_forward():
    """With p=0 the MC path is the deterministic forward."""
    case = Case("edge_N200_T3_sep_p0")
    H, _, arrays = case.inputs()
    prm = mcdo_ref.HeadParams(arrays)
    kF, kA = case.masks()
    assert kF.all() and kA.all()
    Y, A = mcdo_ref.mc_inference(H, prm, kF, kA, 0.0, 0.0)
    Yf, Af = mcdo_ref.forward_eval(H, prm)
    for t in range(case.T):
        np.testing.assert_allclose(Y[t].numpy(), Yf.numpy(), atol=1e-6)
        np.testing.assert_allclose(A[t].numpy(), Af.numpy(), atol=1e-8)


def test_float64_restatement_agrees():
    """fp32 oracle vs its own float64 evaluation (accuracy budget of the fp32 path)."""
    case = Case("cfg2_N512_T30_sep")
    H, _, arrays = case.inputs()
    kF, kA = case.masks()
    Y32, A32 = mcdo_ref.mc_inference(H, mcdo_ref.HeadParams(arrays), kF, kA, case.p_f, case.p_a)
    Y64, A64 = mcdo_ref.mc_inference(H, mcdo_ref.HeadParams(arrays, torch.float64), kF, kA,
                                     case.p_f, case.p_a)
    assert nrel(A32.numpy(), A64.numpy()) < 1e-5
    assert np.max(np.abs(Y32.numpy() - Y64.numpy())) < 1e-5


def test_attention_properties():
    case = Case("small_N64_T4_shared")
    H, _, arrays = case.inputs()
    kF, kA = case.masks()
    Y, A = mcdo_ref.mc_inference(H, mcdo_ref.HeadParams(arrays), kF, kA, case.p_f, case.p_a)
    np.testing.assert_allclose(A.sum(-1).numpy(), 1.0, atol=1e-6)
    assert (A >= 0).all()


def test_permutation_equivariance():
    """Shuffling the bag's instances (the reference shuffles bags, image_patcher.py:131) permutes
    A and leaves Y unchanged when the masks are permuted with them."""
    case = Case("small_N64_T4_sep")
    H, _, arrays = case.inputs()
    kF, kA = case.masks()
    prm = mcdo_ref.HeadParams(arrays)
    perm = np.random.default_rng(0).permutation(case.N)
    Y, A = mcdo_ref.mc_inference(H, prm, kF, kA, case.p_f, case.p_a)
    Yp, Ap = mcdo_ref.mc_inference(H[perm], prm, kF[:, perm], kA[:, :, perm], case.p_f, case.p_a)
    np.testing.assert_allclose(Yp.numpy(), Y.numpy(), atol=1e-5)
    np.testing.assert_allclose(Ap.numpy(), A.numpy()[..., perm], atol=1e-7)
