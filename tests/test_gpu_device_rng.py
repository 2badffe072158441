"""Device mode (dbsde_batch.W == NULL, the path bench.py times) against the
oracle (oracle/philox.py).  Needs an MI355X.

Pins, in order:
  * the device fetch_minibatch (dbsde_brownian): the time grid and W = cumsum(dW)
    are bit-exact restatements of the reference's fetch_minibatch arithmetic;
    the Philox normals match the Random123-pinned oracle to float32 accuracy
    (Box-Muller uses the device's logf / sincospif: rel 2e-6, abs 2e-6);
  * the rollout of device mode consumes exactly those increments: X from
    dbsde_loss_grad(W = NULL) equals the oracle rollout of the device dW bit
    for bit (diagonal, Cholesky-correlated and Heston path kernels);
  * sharding: a rank's paths [path0, path0 + M) draw exactly the single-device
    increments of those paths;
  * the correlated increments equal L (sqrt(dt) z) of the oracle (fp64 einsum)
    within fp32 accumulation error.
"""
import numpy as np
import pytest
import torch

from conftest import load_pkg
from oracle import philox as ph

pytestmark = pytest.mark.gpu

T = 1.0


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


def solver(pkg, dev, D, spec, layers=None, mode="NAIS-Net"):
    layers = layers or [D + 1, 16, 16, 16, 16, 1]
    return pkg.NativeSolver(mode, layers, "Sine", spec, T, dev)


BSB = dict(sig_a=0.4, phi_r=0.05, phi_c=1.0, g="sumsq")
BASKET = dict(mu_a=0.05, sig_a=0.2, phi_r=0.05, phi_c=0.0, g="call_mean", strike=1.0)


def device_X(pkg, dev, s, M, N, Xi, seed, path0=0):
    params = torch.zeros(s.nparams, device=dev)
    X = torch.empty(M * (N + 1) * s.D, device=dev)
    loss = torch.empty(1, device=dev)
    s.loss_grad(params, M, N, torch.as_tensor(Xi, dtype=torch.float32).to(dev).contiguous(), seed=seed,
                path0=path0, loss=loss, X=X)
    torch.cuda.synchronize()
    return X.cpu().numpy().reshape(M, N + 1, s.D)


@pytest.mark.parametrize("N", [5, 8, 50])
def test_fetch_grid_and_W(pkg, dev, N):
    s = solver(pkg, dev, 4, pkg.ProblemSpec(**BSB))
    M = 8
    t, dW = s.brownian(M, N, seed=11, increments=True)
    t2, W = s.brownian(M, N, seed=11)
    torch.cuda.synchronize()
    t, dW, W = t.cpu().numpy(), dW.cpu().numpy(), W.cpu().numpy()
    np.testing.assert_array_equal(t, np.broadcast_to(ph.time_grid(N, T), (M, N + 1)))
    np.testing.assert_array_equal(t2.cpu().numpy(), t)
    np.testing.assert_array_equal(W, ph.brownian_W(dW))        # fp64 cumsum, cast
    ref = ph.increments(11, 0, 0, M, N, 4, T)
    np.testing.assert_allclose(dW, ref, rtol=2e-6, atol=2e-6)


def test_increments_are_standard_normal(pkg, dev):
    s = solver(pkg, dev, 100, pkg.ProblemSpec(**BSB), layers=[101, 110, 110, 110, 110, 1])
    _, dW = s.brownian(1024, 50, seed=3, increments=True)
    z = dW.cpu().numpy().reshape(-1) / np.sqrt(T / 50)
    assert abs(z.mean()) < 5e-3 and abs(z.std() - 1) < 5e-3


def test_shard_draws_global_paths(pkg, dev):
    s = solver(pkg, dev, 4, pkg.ProblemSpec(**BSB))
    _, full = s.brownian(16, 9, seed=5, increments=True)
    _, part = s.brownian(8, 9, seed=5, path0=8, increments=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(full.cpu().numpy()[8:], part.cpu().numpy())


@pytest.mark.parametrize("D,spec", [(4, BSB), (100, BSB), (8, BASKET)], ids=["bsb4", "bsb100", "basket8"])
def test_device_rollout_consumes_the_drawn_increments(pkg, dev, D, spec):
    s = solver(pkg, dev, D, pkg.ProblemSpec(**spec), layers=[D + 1, 16, 16, 16, 16, 1])
    M, N = 32, 50
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    _, dW = s.brownian(M, N, seed=9, increments=True)
    X = device_X(pkg, dev, s, M, N, Xi, seed=9)
    ref = ph.rollout(Xi, dW.cpu().numpy(), T, spec.get("mu_a", 0.0), spec.get("sig_a", 0.0), 0.0)
    np.testing.assert_array_equal(X, ref)
    # path0 shard of the same draw
    Xs = device_X(pkg, dev, s, 16, N, Xi, seed=9, path0=16)
    np.testing.assert_array_equal(Xs, X[16:])


@pytest.mark.parametrize("D", [5, 100])
def test_correlated_device_mode(pkg, dev, D):
    """with_corr...py:339-341: dW = L (sqrt(dt) z), L staged in LDS (rollout_corr_kernel)."""
    rs = np.random.RandomState(D)
    A = rs.normal(size=(D, D))
    C = A @ A.T + D * np.eye(D)
    d = np.sqrt(np.diag(C))
    L = np.linalg.cholesky(C / np.outer(d, d))
    s = solver(pkg, dev, D, pkg.ProblemSpec(**BASKET), layers=[D + 1, 16, 16, 16, 16, 1])
    s.set_corr(L)
    M, N = 24, 10
    _, dW = s.brownian(M, N, seed=4, increments=True)
    dW = dW.cpu().numpy()
    ref = ph.increments(4, 0, 0, M, N, D, T, L=L.astype(np.float32))
    scale = np.abs(ref).max()
    np.testing.assert_allclose(dW, ref, rtol=0, atol=2e-6 * scale * np.sqrt(D))
    Xi = np.ones((1, D))
    X = device_X(pkg, dev, s, M, N, Xi, seed=4)
    np.testing.assert_array_equal(X, ph.rollout(Xi, dW, T, 0.05, 0.2, 0.0))
    s.set_corr(None)
    _, dWu = s.brownian(M, N, seed=4, increments=True)
    np.testing.assert_allclose(dWu.cpu().numpy(), ph.increments(4, 0, 0, M, N, D, T), rtol=2e-6, atol=2e-6)


@pytest.mark.parametrize("k", [1, 50])
def test_heston_device_mode(pkg, dev, k):
    spec = pkg.ProblemSpec(kind="heston", mu_a=0.05, phi_r=0.05, g="call_mean", strike=1.0, g_cols=k, u_clamp=True,
                           q3=False, kappa=2.0, theta=0.2, sigma=0.3, rho=0.8)
    s = pkg.NativeSolver("Naisnet", [1 + 2 * k, 16, 16, 16, 16, 1], "Sine", spec, T, dev)
    assert s.nb == k
    M, N = 16, 20
    Xi = np.concatenate([np.ones((1, k)), np.full((1, k), 0.2)], 1)
    _, dW = s.brownian(M, N, seed=2, increments=True)
    dW = dW.cpu().numpy()
    np.testing.assert_allclose(dW, ph.increments(2, 0, 0, M, N, k, T), rtol=2e-6, atol=2e-6)
    X = device_X(pkg, dev, s, M, N, Xi, seed=2)
    Xr, _ = ph.heston_rollout(Xi, dW, T)
    np.testing.assert_array_equal(X, Xr)


def test_prefetched_rollout_is_the_same_step(pkg, dev):
    """dbsde_prefetch (the next iteration's rollout on the library's prefetch
    stream, overlapping the current one): a loss_grad that consumes a
    prefetched batch returns bit-identical X, loss and gradient to one that
    rolls out itself; a mismatching batch (other seed) is rolled out as usual;
    two batches may be pending at once; a width-110 NAIS-Net (split-bf16
    kernels) and the Cholesky-correlated path kernel both take this route."""
    D, M, N = 100, 128, 10
    rs = np.random.RandomState(3)
    L = np.linalg.cholesky(np.corrcoef(rs.normal(size=(D, 3 * D))) + 1e-3 * np.eye(D)).astype(np.float32)
    for corr in (False, True):
        s = solver(pkg, dev, D, pkg.ProblemSpec(**BASKET), layers=[D + 1] + 4 * [110] + [1])
        if corr:
            s.set_corr(L)
        params = torch.from_numpy(rs.normal(scale=0.05, size=s.nparams).astype(np.float32)).to(dev)
        Xi = torch.ones(D, device=dev)

        def step(seed):
            X = torch.empty(M * (N + 1) * D, device=dev)
            grad, loss = torch.empty_like(params), torch.empty(1, device=dev)
            s.loss_grad(params, M, N, Xi, seed=seed, grad=grad, loss=loss, X=X)
            torch.cuda.synchronize()
            return X.cpu().numpy(), float(loss), grad.cpu().numpy()

        ref = {k: step(k) for k in (5, 6, 7)}
        s.prefetch(M, N, Xi, seed=5)
        s.prefetch(M, N, Xi, seed=6)            # two pending
        got5 = step(5)
        s.prefetch(M, N, Xi, seed=9)            # replaced below: seed 7 is not the prefetched one
        got7 = step(7)
        got6 = step(6)
        for a, b in ((got5, ref[5]), (got6, ref[6]), (got7, ref[7])):
            np.testing.assert_array_equal(a[0], b[0])
            assert a[1] == b[1]
            np.testing.assert_array_equal(a[2], b[2])
