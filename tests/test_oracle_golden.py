"""The oracle (CPU restatement) against golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import fbsnn_ref as fr
from oracle import timeparallel as tp

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
G1 = sorted(p for p in glob.glob(os.path.join(GOLDEN, "g1_*.npz")) if "train_" not in p)
TRAIN = sorted(glob.glob(os.path.join(GOLDEN, "g1_train_*.npz")))


def _load(p):
    z = np.load(p)
    return {k: z[k] for k in z.files}


def _heston(g):
    return dict(kappa=float(g["kappa"]), theta=float(g["theta"]), sigma=float(g["sigma"]), rho=float(g["rho"]),
                v0=float(g["v0"]), payoff=str(g["payoff"]))


@pytest.mark.parametrize("path", G1, ids=[os.path.basename(p)[3:-4] for p in G1])
def test_restatement_matches_reference(path):
    """fp32 autograd restatement == reference run (same params, t, W)."""
    g = _load(path)
    layers = [int(v) for v in g["layers"]]
    D, M = layers[0] - 1, int(g["M"])
    torch.set_num_threads(1)
    if str(g["problem"]) == "heston":
        model = fr.build_heston_model(str(g["mode"]), [2] + layers[1:], str(g["activation"]), D // 2)
        fr.set_flat_params(model, g["params"])
        res = fr.heston_loss_and_grads(model, fr.Heston(k=D // 2, **_heston(g)), torch.from_numpy(g["t"]),
                                       torch.from_numpy(g["W"]), g["Xi"], M)
    else:
        model = fr.build_model(str(g["mode"]), layers, str(g["activation"]))
        fr.set_flat_params(model, g["params"])
        prob = fr.make_problem(str(g["problem"]), D)
        res = fr.loss_and_grads(model, prob, torch.from_numpy(g["t"]), torch.from_numpy(g["W"]),
                                torch.from_numpy(g["Xi"]), M, D)
    np.testing.assert_array_equal(res["X"], g["X"])          # the rollout is bit-exact
    np.testing.assert_allclose(res["loss"], g["loss"], rtol=1e-6)
    np.testing.assert_allclose(res["Y"], g["Y"], rtol=1e-6, atol=1e-6)
    if "Z" in g:                                              # full-shape fixtures store no Z
        np.testing.assert_allclose(res["Z"], g["Z"], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(res["used"], g["used"])
    scale = np.abs(g["grad"]).max()
    np.testing.assert_allclose(res["grad"], g["grad"], rtol=0, atol=1e-5 * scale)


@pytest.mark.parametrize("path", G1, ids=[os.path.basename(p)[3:-4] for p in G1])
def test_timeparallel_matches_reference(path):
    """The hand-derived time-parallel algorithm (fp64) reproduces the
    reference's fp32 loss / Z / gradient to fp32 accuracy."""
    g = _load(path)
    layers = [int(v) for v in g["layers"]]
    heston = str(g["problem"]) == "heston"
    out = tp.loss_grad(g["params"].astype(np.float64), str(g["mode"]), layers, str(g["activation"]),
                       str(g["problem"]), g["t"].astype(np.float64), g["W"].astype(np.float64),
                       (g["Xi_full"] if heston else g["Xi"]).astype(np.float64),
                       heston=_heston(g) if heston else None)
    np.testing.assert_allclose(out["loss"], g["loss"], rtol=2e-5)
    np.testing.assert_allclose(out["X"], g["X"], rtol=1e-6, atol=1e-6 * max(1.0, np.abs(g["X"]).max()))
    np.testing.assert_allclose(out["Y"], g["Y"], rtol=1e-5, atol=1e-5)
    if "Z" in g:
        np.testing.assert_allclose(out["Z"], g["Z"], rtol=1e-4, atol=1e-5)
    used = g["used"]
    scale = np.abs(g["grad"]).max()
    np.testing.assert_allclose(out["grad"][used], g["grad"][used], rtol=0, atol=1e-4 * scale)


@pytest.mark.parametrize("path", TRAIN, ids=[os.path.basename(p)[3:-4] for p in TRAIN])
def test_restated_training_matches_reference(path):
    """Reference train() for 10 iterations (fresh Adam, clip per file)."""
    g = _load(path)
    layers = [int(v) for v in g["layers"]]
    D, M, N = layers[0] - 1, int(g["M"]), int(g["N"])
    torch.set_num_threads(1)
    if str(g["problem"]) == "heston":
        model = fr.build_heston_model(str(g["mode"]), [2] + layers[1:], str(g["activation"]), D // 2)
        fr.set_flat_params(model, g["params0"])
        np.random.seed(int(g["batch_seed"]))
        fr.heston_train(model, fr.Heston(k=D // 2, **_heston(g)), g["Xi"], M, N, float(g["T"]), int(g["iters"]),
                        float(g["lr"]), Mm=float(g["Mm"]))
        np.testing.assert_allclose(fr.flat_params(model), g["params1"], rtol=0, atol=2e-6)
        return
    model = fr.build_model(str(g["mode"]), layers, str(g["activation"]))
    fr.set_flat_params(model, g["params0"])
    prob = fr.make_problem(str(g["problem"]), D)
    np.random.seed(int(g["batch_seed"]))
    Mm = float(g["Mm"])
    name = os.path.basename(path)
    corr = "corr_" in name
    L = np.linalg.cholesky(g["corr"]) if corr else None
    lbfgs = "lbfgs" in name
    fr.train(model, prob, g["Xi"], M, N, D, float(g["T"]), int(g["iters"]), float(g["lr"]),
             clip=bool(g["clip"]) if "clip" in g else True, Mm=None if Mm < 0 else Mm,
             start_it=int(g["start_iteration"]) if "start_iteration" in g else 0, L=L,
             schedule="corr" if corr else "nd", optimizer="LBFGS" if lbfgs else "Adam")
    # LBFGS (60 closure evaluations at lr 0.05) amplifies the summation-order
    # differences of the restatement
    np.testing.assert_allclose(fr.flat_params(model), g["params1"], rtol=0, atol=2e-4 if lbfgs else 2e-6)


def test_n_schedule_quirk():
    """Mm = 50**(1/5) gives N = 3 until it=4000, then 5, 11, 23, 51."""
    Mm = 50 ** (1 / 5)
    got = [fr.n_schedule(it, Mm, 50) for it in (0, 3999, 4000, 8000, 12000, 16000, 19999, 20000)]
    assert got == [3, 3, 5, 11, 23, 51, 51, 50]


def test_bsb_known_answer():
    """u(0, X0) = exp(0.21) * 62.5 = 77.1049 for Xi = [1, 0.5]*50 (DeepBSDE.py:345-349)."""
    Xi = np.array([1.0, 0.5] * 50)[None, :]
    assert abs(fr.bsb_u_exact(0.0, Xi)[0, 0] - 77.1049) < 1e-4
