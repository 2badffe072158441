"""The rest of the FBSNN surface on the HIP path: the optimizer menu against
torch.optim, checkpoint interop with the reference's save format, predict /
PredictionGenerator against the reference's outputs, the exact-solution
evaluators and the HJB Monte-Carlo comparator, and the BASELINE configs 3-5 at
their real shapes.  Needs an MI355X."""
import glob
import math
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_pkg
from oracle import philox as ph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


def _load(name):
    z = np.load(os.path.join(GOLDEN, name))
    return {k: z[k] for k in z.files}


def bsb_model(pkg, dev, g):
    layers = [int(v) for v in g["layers"]]
    m = pkg.BlackScholesBarenblatt(g["Xi"], float(g["T"]), int(g["M"]), int(g["N"]), layers[0] - 1, layers,
                                   str(g["mode"]), str(g["activation"]), device=dev)
    m.params.copy_(torch.from_numpy(g["params"]).to(dev))
    return m


# --------------------------------------------------------------------------- optimizers
@pytest.mark.parametrize("name", ["Adam", "AdamW", "SGD", "RMSprop", "Adagrad", "Adamax", "Adadelta", "ASGD"])
def test_optimizer_matches_torch(pkg, dev, name):
    """Four steps of the native optimizer (clip 1.0 first, nd_BSPDE_case.py:383-384)
    == torch.optim.<name>(params, lr) + clip_grad_norm_ on the CPU, same grads."""
    g = _load("g1_deep_bsb_NAIS-Net_Sine.npz")
    m = bsb_model(pkg, dev, g)
    m.clip_max_norm = 1.0
    lr = 1e-2
    opt = m.new_optimizer_state(name, lr)
    ref = torch.from_numpy(g["params"]).clone().requires_grad_(True)
    topt = getattr(torch.optim, name)([ref], lr=lr)
    used = torch.from_numpy(g["used"])
    rs = np.random.RandomState(0)
    for _ in range(4):
        grad = torch.from_numpy(g["grad"] * rs.uniform(0.5, 2.0)).float() * used
        m.grad.copy_(grad.to(dev))
        m._update(opt)
        topt.zero_grad()
        ref.grad = grad.clone()
        torch.nn.utils.clip_grad_norm_([ref], max_norm=1.0)
        topt.step()
    got = m.params.cpu().numpy()
    want = ref.detach().numpy()
    np.testing.assert_allclose(got[g["used"]], want[g["used"]], rtol=0, atol=2e-6 * max(1.0, np.abs(want).max()))
    if name == "AdamW":
        assert not np.allclose(got, g["params"])        # the decoupled decay acted


def test_nan_loss_skips_the_update(pkg, dev):
    """heston_dnnpde.py:409-411: a non-finite loss leaves params and moments untouched."""
    g = _load("g1_deep_bsb_NAIS-Net_Sine.npz")
    m = bsb_model(pkg, dev, g)
    opt = m.new_optimizer_state("Adam", 1e-3)
    m.grad.copy_(torch.from_numpy(g["grad"]).to(dev))
    loss = torch.tensor([float("nan")], device=dev)
    before = m.params.clone()
    m._update(opt, skip_loss=loss)
    torch.cuda.synchronize()
    assert torch.equal(before, m.params) and float(opt["m"].abs().max()) == 0.0


# --------------------------------------------------------------------------- checkpoints / predict
def test_checkpoint_round_trip_reference_format(pkg, dev, tmp_path):
    """A checkpoint in the reference's save format (nd_BSPDE_case.py:445-456,
    training_loss as numpy float64 from np.mean) loads through load_model with
    the weights-only loader, reproduces the fixture's loss, and saves back."""
    g = _load("g1_nd_call_Naisnet_Sine.npz")
    layers = [int(v) for v in g["layers"]]
    D = layers[0] - 1
    m = pkg.CallOption(g["Xi"], float(g["T"]), int(g["M"]), int(g["N"]), D, 5.0, layers, str(g["mode"]),
                       str(g["activation"]), device=dev)
    donor = pkg.CallOption(g["Xi"], float(g["T"]), int(g["M"]), int(g["N"]), D, 5.0, layers, str(g["mode"]),
                           str(g["activation"]), device=dev)
    donor.params.copy_(torch.from_numpy(g["params"]).to(dev))
    sd = {k: v.detach().cpu().clone() for k, v in donor.model.state_dict().items()}
    path = str(tmp_path / "ref.pt")
    torch.save({"model_state_dict": sd, "training_loss": [np.mean(np.array([1.5, 2.5])), np.float64(0.25)],
                "iteration": [0, 100]}, path)
    m.load_model(path)
    assert m.training_loss == [2.0, 0.25] and m.iteration == [0, 100]
    loss, X, Y, _ = m.loss_function(torch.from_numpy(g["t"]).to(dev), torch.from_numpy(g["W"]).to(dev), m.Xi)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-4)
    path2 = str(tmp_path / "ours.pt")
    m.save_model(path2)
    m2 = pkg.CallOption(g["Xi"], float(g["T"]), int(g["M"]), int(g["N"]), D, 5.0, layers, str(g["mode"]),
                        str(g["activation"]), device=dev)
    m2.load_model(path2)
    torch.testing.assert_close(m2.params, m.params, rtol=0, atol=0)


def test_predict_matches_reference_outputs(pkg, dev):
    """nd_BSPDE_case.py:412-443: predict(Xi, t, W) -> (X, Y) == the reference's."""
    g = _load("g1_deep_bsb_NAIS-Net_Sine.npz")
    m = bsb_model(pkg, dev, g)
    X, Y = m.predict(g["Xi"], g["t"], g["W"])
    np.testing.assert_array_equal(X.cpu().numpy(), g["X"])
    np.testing.assert_allclose(Y.cpu().numpy(), g["Y"], rtol=0, atol=1e-4 * max(1.0, np.abs(g["Y"]).max()))
    assert m.M == int(g["M"])


def test_heston_predict_returns_S_v_Y(pkg, dev):
    g = _load("g1_heston_Naisnet_Sine.npz")
    layers = [int(v) for v in g["layers"]]
    m = pkg.HestonFBSNN(g["Xi"], 1.0, int(g["M"]), int(g["N"]), 1, 5.0, [2] + layers[1:], "Naisnet", "Sine",
                        device=dev)
    m.params.copy_(torch.from_numpy(g["params"]).to(dev))
    S, v, Y = m.predict(g["Xi"], g["t"], g["W"])
    # 1-ulp torch (MKL vsSqrt) near-tie differences propagate, see test_gpu_parity.py
    np.testing.assert_allclose(S.cpu().numpy(), g["X"][:, :, 0:1], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(v.cpu().numpy(), g["X"][:, :, 1:2], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Y.cpu().numpy(), g["Y"], rtol=0, atol=1e-4 * max(1.0, np.abs(g["Y"]).max()))


def test_prediction_generator(pkg, dev):
    """nd_BSPDE_case.py:543-584: 16 batches from np.random.seed(42), concatenated."""
    g = _load("g1_deep_bsb_NAIS-Net_Sine.npz")
    m = bsb_model(pkg, dev, g)
    t, W0, X, Y = pkg.PredictionGenerator(m, g["Xi"], 16).generate_predictions()
    M, N = int(g["M"]), int(g["N"])
    assert X.shape == (16 * M, N + 1, X.shape[2]) and Y.shape == (16 * M, N + 1, 1) and t.shape[0] == 16 * M
    np.random.seed(42)
    t1, W1 = m.fetch_minibatch()
    np.testing.assert_array_equal(W0.cpu().numpy(), W1.cpu().numpy())
    X1, Y1 = m.predict(g["Xi"], t1, W1)
    np.testing.assert_array_equal(X[:M], X1.cpu().numpy())


# --------------------------------------------------------------------------- evaluators
def _ncdf(x):
    from scipy.stats import norm
    return norm.cdf(x)


def test_exact_evaluators_match_reference_formulas(pkg, dev):
    rs = np.random.RandomState(1)
    R, D, T = 64, 5, 1.0
    X = rs.uniform(0.5, 1.5, size=(R, D)).astype(np.float32)
    t = rs.uniform(0.0, 1.0, size=R).astype(np.float32)
    t[:4] = T                                  # at maturity: payoff and 0 / 1 deltas
    Xt, tt = torch.from_numpy(X).to(dev), torch.from_numpy(t).to(dev)
    X64, tau = X.astype(np.float64), T - t.astype(np.float64)
    # BSB u_exact (DeepBSDE.py:345-349)
    u, _ = pkg.exact("bsb", tt, Xt, T, [0.05, 0.4])
    np.testing.assert_allclose(u.cpu().numpy()[:, 0], np.exp(0.21 * tau) * np.sum(X64 ** 2, 1), rtol=1e-6)
    # Black-Scholes call per coordinate (nd_BSPDE_case.py:587-618)
    r, sig, K = 0.05, 0.2, 1.0
    p, d = pkg.exact("bs_call", tt, Xt, T, [r, sig, K])
    with np.errstate(divide="ignore", invalid="ignore"):
        tau2 = np.repeat(tau[:, None], D, 1)
        d1 = (np.log(X64 / K) + (r + 0.5 * sig ** 2) * tau2) / (sig * np.sqrt(tau2))
        d2 = d1 - sig * np.sqrt(tau2)
        pr = np.where(tau2 > 0, X64 * _ncdf(d1) - K * np.exp(-r * tau2) * _ncdf(d2), np.maximum(X64 - K, 0))
        dr = np.where(tau2 > 0, _ncdf(d1), (X64 > K).astype(float))
    np.testing.assert_allclose(p.cpu().numpy(), pr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d.cpu().numpy(), dr, rtol=1e-5, atol=1e-6)
    # basket: averaged sigma on mean(x) (with_corr...py:663-700) and mean of per-asset calls
    p, _ = pkg.exact("basket_avg", tt, Xt, T, [r, sig, K])
    Sa, sa = X64.mean(1), sig / np.sqrt(D)
    with np.errstate(divide="ignore", invalid="ignore"):
        d1 = (np.log(Sa / K) + (r + 0.5 * sa ** 2) * tau) / (sa * np.sqrt(tau))
        pa = np.where(tau > 0, Sa * _ncdf(d1) - K * np.exp(-r * tau) * _ncdf(d1 - sa * np.sqrt(tau)),
                      np.maximum(Sa - K, 0))
    np.testing.assert_allclose(p.cpu().numpy()[:, 0], pa, rtol=1e-5, atol=1e-6)
    p, _ = pkg.exact("basket_mean", tt, Xt, T, [r, sig, K])
    np.testing.assert_allclose(p.cpu().numpy()[:, 0], pr.mean(1), rtol=1e-5, atol=1e-6)


def test_hjb_mc_matches_oracle_on_the_same_draws(pkg, dev):
    """dbsde_hjb_mc == oracle/philox.hjb_value (same Philox draws, fp64 sums)."""
    rs = np.random.RandomState(2)
    P, D, mc = 4, 10, 4096
    X = rs.normal(size=(P, D)).astype(np.float32)
    t = np.array([0.0, 0.25, 0.5, 1.0], np.float32)
    u = pkg.hjb_mc(torch.from_numpy(t).to(dev), torch.from_numpy(X).to(dev), 1.0, mc=mc, seed=7).cpu().numpy()
    ref = ph.hjb_value(t, X, 1.0, mc, 7)
    np.testing.assert_allclose(u, ref, rtol=2e-5, atol=2e-6)


def test_hjb_mc_known_value(pkg, dev):
    """hjb_implement.py:1088-1095 at D = 100, x = 0, t = 0 with 10^5 samples,
    against the reference's numpy formula on numpy draws (MC error ~1e-3)."""
    D, mc = 100, 10 ** 5
    u = float(pkg.hjb_mc(torch.zeros(1, device=dev), torch.zeros(1, D, device=dev), 1.0, mc=mc, seed=1))
    rs = np.random.RandomState(0)
    W = rs.normal(size=(mc, 1, D))
    g = np.log(0.5 + 0.5 * np.sum((np.sqrt(2.0) * W) ** 2, axis=2, keepdims=True))
    ref = float(-np.log(np.mean(np.exp(-g), axis=0)))
    assert abs(u - ref) < 5e-3, (u, ref)


# --------------------------------------------------------------------------- configs 3-5 at real shapes
def _device_steps(m, k=2, name="Adam"):
    opt = m.new_optimizer_state(name, 1e-3)
    losses = [float(m.device_step(opt, 1e-3, seed=s)) for s in range(k)]
    torch.cuda.synchronize()
    return losses


def test_config3_basket_correlated_device_step(pkg, dev):
    """BASELINE config 3 on one GPU: 100-D basket, Cholesky-correlated device
    increments (Q10 matrix), Naisnet-ReLU [101,110x4,1], M=4096."""
    np.random.seed(0)
    torch.manual_seed(0)
    D = 100
    m = pkg.BasketCallOption(np.ones((1, D)), 1.0, 4096, 50, D, 50 ** 0.2, [D + 1] + 4 * [110] + [1], "Naisnet",
                             "ReLU", "random_correlation", device=dev)
    m.N = 50
    losses = _device_steps(m)
    assert all(np.isfinite(losses)) and torch.isfinite(m.params).all()


def test_config4_hjb_fc256(pkg, dev):
    """BASELINE config 4 on one GPU: 100-D HJB, FC-Sine [101,256x4,1], M=2048, N=20."""
    torch.manual_seed(0)
    D = 100
    m = pkg.HamiltonJacobiBellman(np.zeros((1, D)), 1.0, 2048, 20, D, [D + 1] + 4 * [256] + [1], "FC", "Sine",
                                  device=dev)
    losses = _device_steps(m)
    assert all(np.isfinite(losses)) and torch.isfinite(m.params).all()


def test_config5_heston_50_assets(pkg, dev):
    """BASELINE config 5 on one GPU: 50-asset Heston (state 100), M=1024, N=100,
    Naisnet-Sine [101,110x4,1], two device-mode training steps stay finite.
    Its numbers are checked in tests/test_gpu_round3.py: k = 3 / 50 against the
    oracle's per-asset restatement (parity unpinned beyond one asset: the
    reference has k = 1 only) and the fused vs per-layer paths at this shape."""
    torch.manual_seed(0)
    k = 50
    m = pkg.HestonFBSNN(np.ones((1, k)), 1.0, 1024, 100, k, None, [k + 1] + 4 * [110] + [1], "Naisnet", "Sine",
                        device=dev)
    losses = _device_steps(m)
    assert all(np.isfinite(losses)) and torch.isfinite(m.params).all()
