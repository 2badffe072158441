"""Configs 3, 4 and 5 at their full BASELINE shapes against the oracle (needs
an MI355X): until round 5 these shapes were checked only against the build
itself (fused vs per-layer kernels, a batch vs the sum of its halves,
tests/test_gpu_round3.py); here the HIP loss, X, Y, Z and gradient of one
step are compared with oracle/fbsnn_ref.py -- the restatement pinned to the
reference's own fixtures -- run on the host with the same t / W:

  * config 3: 100-D basket, Cholesky-correlated increments (the Q10 recipe),
    Naisnet-ReLU [101,110x4,1], M = 4096, N = 50 (with_corr...py:316-353,
    561-616);
  * config 4: 100-D HJB, FC-Sine [101,256x4,1], M = 2048, N = 20
    (hjb_implement.py:590-604);
  * config 5: 50-asset Heston (state 100), Naisnet-Sine [101,110x4,1],
    M = 1024, N = 100 (heston_dnnpde.py:519-659; parity unpinned beyond one
    asset, as tests/test_gpu_round3.py says).

Tolerances as tests/test_gpu_parity.py: X bit-exact, loss rel 1e-4, Y / Z abs
1e-4 max|ref|, gradient abs 2e-4 max|ref grad|, with two full-shape
adjustments:
  * ReLU (config 3): Z = grad_x u has a jump wherever a pre-activation
    crosses 0, so among 2e7 Z elements a few rows whose pre-activation lies
    within fp32 rounding of 0 take the other branch in one of the two
    summation orders; at most 1e-5 of the Z elements may exceed the
    tolerance (observed 9e-6);
  * Heston (config 5): the host's float32 torch.sqrt (MKL vsSqrt) is not
    correctly rounded at near-ties and the kernel's is, and over N = 100
    variance steps a one-ulp difference grows; the oracle runs with sqrt
    computed in fp64 and rounded once to fp32 (the correctly rounded fp32
    sqrt), after which X is compared bit for bit like the other rollouts."""
import numpy as np
import pytest
import torch

from conftest import load_pkg
from oracle import fbsnn_ref as fr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


def _native(s, params, M, N, D, Xi, t, W, dev):
    out = dict(loss=torch.empty(1, device=dev), X=torch.empty(M * (N + 1) * D, device=dev),
               Y=torch.empty(M * (N + 1), device=dev), Z=torch.empty(M * (N + 1) * D, device=dev))
    grad = torch.empty_like(params)
    s.loss_grad(params, M, N, torch.as_tensor(Xi, dtype=torch.float32).to(dev).contiguous(),
                t=torch.as_tensor(t).float().to(dev).reshape(M, N + 1).contiguous(),
                W=torch.as_tensor(W).float().to(dev).contiguous(), grad=grad, **out)
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in out.items()}
    r["grad"] = grad.cpu().numpy()
    r["X"] = r["X"].reshape(M, N + 1, D)
    r["Z"] = r["Z"].reshape(M, N + 1, D)
    r["Y"] = r["Y"].reshape(M, N + 1, 1)
    return r


def _grid(M, N):
    return np.tile(np.concatenate([[0.0], np.cumsum(np.full(N, 1.0 / N))]), (M, 1)).astype(np.float32)


def _check(r, ref, z_kink_frac=0.0):
    np.testing.assert_array_equal(r["X"], ref["X"])
    np.testing.assert_allclose(r["loss"][0], ref["loss"], rtol=1e-4)
    np.testing.assert_allclose(r["Y"], ref["Y"], rtol=0, atol=1e-4 * max(1.0, np.abs(ref["Y"]).max()))
    ztol = 1e-4 * max(1.0, np.abs(ref["Z"]).max())
    if z_kink_frac > 0.0:
        bad = np.abs(r["Z"] - ref["Z"]) > ztol
        assert bad.mean() <= z_kink_frac, (int(bad.sum()), bad.size)
    else:
        np.testing.assert_allclose(r["Z"], ref["Z"], rtol=0, atol=ztol)
    used = ref["used"]
    np.testing.assert_allclose(r["grad"][used], ref["grad"][used], rtol=0, atol=2e-4 * np.abs(ref["grad"]).max())


def _diag_case(pkg, dev, kind, mode, layers, act, spec, M, N, seed, Xi, L=None):
    D = layers[0] - 1
    rs = np.random.RandomState(seed)
    dw = np.sqrt(1.0 / N) * rs.normal(size=(M, N, D))
    if L is not None:
        dw = np.einsum("ij,mnj->mni", L, dw)
    W = np.concatenate([np.zeros((M, 1, D)), np.cumsum(dw, 1)], 1).astype(np.float32)
    t = _grid(M, N)
    torch.manual_seed(seed)
    model = fr.build_model(mode, layers, act)
    params = fr.flat_params(model)
    torch.set_num_threads(16)
    ref = fr.loss_and_grads(model, fr.make_problem(kind, D), torch.from_numpy(t)[:, :, None],
                            torch.from_numpy(W), torch.as_tensor(Xi, dtype=torch.float32), M, D)
    s = pkg.NativeSolver(mode, layers, act, spec, 1.0, dev)
    r = _native(s, torch.from_numpy(params).to(dev), M, N, D, Xi, t, W, dev)
    return r, ref, s


def test_config3_full_shape_matches_oracle(pkg, dev):
    D = 100
    np.random.seed(3)
    L = np.linalg.cholesky(pkg.FBSNN._random_corr(D, False))      # the Q10 recipe (with_corr...py:187-212)
    spec = pkg.ProblemSpec(mu_a=0.05, sig_a=0.20, phi_r=0.05, phi_c=0.0, g="call_mean", strike=1.0)
    r, ref, s = _diag_case(pkg, dev, "basket", "Naisnet", [D + 1] + 4 * [110] + [1], "ReLU", spec, 4096, 50, 3,
                           np.ones((1, D)), L)
    assert s.matrix_form & 1, "config 3 should run the fused kernels"
    _check(r, ref, z_kink_frac=1e-5)


def test_config4_full_shape_matches_oracle(pkg, dev):
    D = 100
    spec = pkg.ProblemSpec(sig_b=float(np.sqrt(2.0)), phi_zz=1.0, g="log")
    r, ref, s = _diag_case(pkg, dev, "hjb", "FC", [D + 1] + 4 * [256] + [1], "Sine", spec, 2048, 20, 4,
                           np.zeros((1, D)))
    assert s.matrix_form & 1, "config 4 should run the fused width-256 kernels"
    _check(r, ref)


def test_config5_full_shape_matches_oracle(pkg, dev):
    k, M, N = 50, 1024, 100
    layers = [1 + 2 * k] + 4 * [110] + [1]
    torch.manual_seed(5)
    model = fr.build_heston_model("Naisnet", [2] + layers[1:], "Sine", k)
    params = fr.flat_params(model)
    np.random.seed(5)
    t, W = fr.fetch_minibatch(M, N, k, 1.0)
    Xi = np.ones((1, k))
    torch.set_num_threads(16)
    sqrt32 = torch.sqrt
    torch.sqrt = lambda x: sqrt32(x.double()).float() if x.dtype == torch.float32 else sqrt32(x)
    try:
        ref = fr.heston_loss_and_grads(model, fr.Heston(k=k, payoff="discontinuous"), t, W, Xi, M)
    finally:
        torch.sqrt = sqrt32
    spec = pkg.ProblemSpec(kind="heston", mu_a=0.05, phi_r=0.05, g="call_mean", strike=1.0, g_alpha=10.0, g_cols=k,
                           u_clamp=True, q3=False, kappa=2.0, theta=0.2, sigma=0.3, rho=0.8)
    s = pkg.NativeSolver("Naisnet", layers, "Sine", spec, 1.0, dev)
    assert s.nb == k
    xi_full = np.concatenate([Xi, np.full((1, k), 0.2)], 1)
    r = _native(s, torch.from_numpy(params).to(dev), M, N, 2 * k, xi_full, t.squeeze(-1), W, dev)
    assert s.matrix_form & 1, "config 5 should run the fused kernels"
    _check(r, ref)
