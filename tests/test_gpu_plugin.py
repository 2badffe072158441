"""The reference's plugin API on the HIP path (needs an MI355X): FBSNN
subclasses defined the reference's way -- overriding phi_tf / g_tf / mu_tf /
sigma_tf (nd_BSPDE_case.py:458-500), no problem_spec() -- and subclasses whose
overrides disagree with the spec they inherit run their own coefficient
methods (generic.py: rollout and residuals in torch on the device, u / Z and
the whole network backward through dbsde_net_u / dbsde_net_u_vjp), checked
against the oracle's autograd of the reference loss (oracle/fbsnn_ref.py)
on a problem ProblemSpec cannot express.

Tolerances (as tests/test_gpu_parity.py): loss rel 1e-4; gradient abs
2e-4 max|g|; Y, Z abs 1e-4 max(1, |ref|); parameters after 10 train()
iterations abs 5e-5; X rel 1e-6 (the rollout is the reference's torch
expression, evaluated by torch on the device)."""
import numpy as np
import pytest
import torch

from conftest import load_pkg
from oracle import fbsnn_ref as fr

pytestmark = pytest.mark.gpu

D, M, N, T = 8, 64, 10, 1.0
LAYERS = [D + 1, 16, 16, 16, 16, 1]


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


class OracleCustom(fr.Problem):
    """mu = 0.05 X (1 + t), sigma = diag(0.2 X + 0.05 t), phi = 0.05 Y + 0.1 |Z|,
    g = |X|^4 / D: time-dependent drift and diffusion, a |Z| driver and a
    quartic payoff -- none of it in the native coefficient table."""

    def mu(self, t, X, Y, Z):
        return 0.05 * X * (1 + t)

    def sigma(self, t, X, Y):
        return torch.diag_embed(0.2 * X + 0.05 * t)

    def phi(self, t, X, Y, Z):
        return 0.05 * Y + 0.1 * torch.sqrt(torch.sum(Z ** 2, dim=1, keepdim=True))

    def g(self, X):
        return torch.sum(X ** 2, dim=1, keepdim=True) ** 2 / self.D


class OracleBSB03(fr.Problem):
    def sigma(self, t, X, Y):
        return 0.3 * torch.diag_embed(X)


def custom_class(pkg):
    class Custom(pkg.FBSNN):
        """The reference's way: the four abstract methods, no problem_spec."""

        def mu_tf(self, t, X, Y, Z):
            return 0.05 * X * (1 + t)

        def sigma_tf(self, t, X, Y):
            return torch.diag_embed(0.2 * X + 0.05 * t)

        def phi_tf(self, t, X, Y, Z):
            return 0.05 * Y + 0.1 * torch.sqrt(torch.sum(Z ** 2, dim=1, keepdim=True))

        def g_tf(self, X):
            return torch.sum(X ** 2, dim=1, keepdim=True) ** 2 / self.D
    return Custom


def _xi():
    return np.random.RandomState(7).uniform(0.5, 1.5, (1, D)).astype(np.float32)


def _oracle_model(m, mode="Naisnet"):
    model = fr.build_model(mode, m.layers, m.activation)
    fr.set_flat_params(model, m.params.detach().cpu())
    return model


def _compare(out, g, ref, used):
    assert float(out["loss"]) == pytest.approx(ref["loss"], rel=1e-4)
    np.testing.assert_allclose(out["X"].cpu().numpy(), ref["X"], rtol=1e-6, atol=1e-6)
    Yr = ref["Y"]
    np.testing.assert_allclose(out["Y"].cpu().numpy(), Yr, rtol=0, atol=1e-4 * max(1.0, np.abs(Yr).max()))
    Zr = ref["Z"]
    np.testing.assert_allclose(out["Z"].cpu().numpy(), Zr, rtol=0, atol=1e-4 * max(1.0, np.abs(Zr).max()))
    gr = ref["grad"]
    got = g.cpu().numpy()
    np.testing.assert_allclose(got[used], gr[used], rtol=0, atol=2e-4 * np.abs(gr).max())


def test_custom_problem_matches_oracle(pkg, dev):
    torch.manual_seed(11)
    m = custom_class(pkg)(_xi(), T, M, N, D, None, LAYERS, "Naisnet", "Sine", device=dev)
    assert not m.native_coefficients and m.generic_reason == "no problem_spec()"
    np.random.seed(12)
    t, W = fr.fetch_minibatch(M, N, D, T)
    Xi = torch.from_numpy(_xi())
    ref = fr.loss_and_grads(_oracle_model(m), OracleCustom(kind="custom", D=D), t, W, Xi, M, D)
    g = torch.empty_like(m.params)
    out = m._run(t.to(dev), W.to(dev), Xi.to(dev), grad=g, want=("X", "Y", "Z"))
    torch.cuda.synchronize()
    _compare(out, g, ref, ref["used"])

    # the reference's own calling convention: loss_function, then loss.backward()
    for p in m.model.parameters():
        p.grad = None
    loss, X, Y, y0 = m.loss_function(t.to(dev), W.to(dev), Xi.to(dev))
    loss.backward()
    got = torch.cat([p.grad.reshape(-1) for p in m.model.parameters() if p.grad is not None])
    want = torch.cat([x.reshape(-1) for x in m._param_grads(g) if x is not None])
    torch.testing.assert_close(got, want, rtol=0, atol=1e-6 * float(want.abs().max()))
    assert float(loss) == pytest.approx(ref["loss"], rel=1e-4)


def test_custom_problem_trains_like_oracle(pkg, dev):
    """Ten reference train() iterations (numpy minibatch stream, clip 1.0,
    Adam) against the oracle's train() from the same initial weights."""
    torch.manual_seed(13)
    m = custom_class(pkg)(_xi(), T, M, N, D, None, LAYERS, "Naisnet", "Sine", device=dev)
    m.log_print = False
    model = _oracle_model(m)
    np.random.seed(21)
    _, min_loss, _ = m.train(10, 1e-3)
    np.random.seed(21)
    losses, _ = fr.train(model, OracleCustom(kind="custom", D=D), _xi(), M, N, D, T, 10, 1e-3, clip=True, Mm=None)
    assert min_loss == pytest.approx(min(losses), rel=1e-4)
    np.testing.assert_allclose(m.params.detach().cpu().numpy(), fr.flat_params(model), rtol=0, atol=5e-5)


def test_overridden_sigma_of_a_spec_problem_is_not_ignored(pkg, dev):
    """class MyBSB(BlackScholesBarenblatt) with sigma = 0.3 diag(X): the
    inherited spec says 0.4, so the override runs (with a warning) and the
    result is the oracle's sigma = 0.3 problem, not the parent's."""

    class MyBSB(pkg.BlackScholesBarenblatt):
        def sigma_tf(self, t, X, Y):
            return 0.3 * torch.diag_embed(X)

    torch.manual_seed(17)
    with pytest.warns(UserWarning, match="sigma_tf"):
        m = MyBSB(_xi(), T, M, N, D, [D + 1, 16, 16, 16, 16, 1], "NAIS-Net", "Sine", device=dev)
    assert not m.native_coefficients
    base = pkg.BlackScholesBarenblatt(_xi(), T, M, N, D, [D + 1, 16, 16, 16, 16, 1], "NAIS-Net", "Sine", device=dev)
    assert base.native_coefficients
    np.random.seed(18)
    t, W = fr.fetch_minibatch(M, N, D, T)
    Xi = torch.from_numpy(_xi())
    model = _oracle_model(m, "NAIS-Net")
    ref03 = fr.loss_and_grads(model, OracleBSB03(kind="bsb", D=D), t, W, Xi, M, D)
    ref04 = fr.loss_and_grads(model, fr.make_problem("bsb", D), t, W, Xi, M, D)
    g = torch.empty_like(m.params)
    out = m._run(t.to(dev), W.to(dev), Xi.to(dev), grad=g, want=("X", "Y", "Z"))
    torch.cuda.synchronize()
    _compare(out, g, ref03, ref03["used"])
    assert abs(float(out["loss"]) - ref04["loss"]) > 1e-3 * abs(ref04["loss"])


def test_state_dependent_drift_is_rejected(pkg, dev):
    class YDrift(custom_class(pkg)):
        def mu_tf(self, t, X, Y, Z):
            return 0.05 * X + 0.01 * Y

    with pytest.raises(ValueError, match="depends on Y or Z"):
        YDrift(_xi(), T, M, N, D, None, LAYERS, "Naisnet", "Sine", device=dev)


def test_generic_device_step(pkg, dev):
    """Throughput mode on the generic path: the device Philox increments
    (dbsde_brownian), the generic loss, the native gradient and update; the
    step's loss equals the loss of the exported batch."""
    torch.manual_seed(19)
    m = custom_class(pkg)(_xi(), T, M, N, D, None, LAYERS, "Naisnet", "Sine", device=dev)
    t, W = m.solver.brownian(M, N, seed=5)
    expect = float(m._run(t, W, m._xi_rows(m.Xi, M), want=())["loss"])
    p0 = m.params.detach().clone()
    opt = m.new_optimizer_state("Adam", 1e-3)
    loss = float(m.device_step(opt, 1e-3, seed=5))
    assert loss == pytest.approx(expect, rel=1e-6)
    assert not torch.equal(p0, m.params)
    for it in range(3):
        assert np.isfinite(float(m.device_step(opt, 1e-3, seed=6 + it)))


@pytest.mark.parametrize("Dg,mode,act", [(1, "Naisnet", "Sine"), (8, "FC", "Tanh"), (8, "Resnet", "Tanh"),
                                         (8, "NAIS-Net", "ReLU")])
def test_custom_problem_other_shapes_match_oracle(pkg, dev, Dg, mode, act):
    """The generic path at D = 1 (the reference's squeeze() broadcast of the
    Y-tilde term, DeepBSDE.py:232-233 / SURVEY Q1) and on the other network
    modes: loss, X / Y / Z and the gradient against the oracle's autograd."""
    layers = [Dg + 1, 16, 16, 16, 16, 1]
    xi = np.random.RandomState(9).uniform(0.5, 1.5, (1, Dg)).astype(np.float32)
    torch.manual_seed(23)
    m = custom_class(pkg)(xi, T, M, N, Dg, None, layers, mode, act, device=dev)
    assert not m.native_coefficients
    np.random.seed(24)
    t, W = fr.fetch_minibatch(M, N, Dg, T)
    Xi = torch.from_numpy(xi)
    ref = fr.loss_and_grads(_oracle_model(m, mode), OracleCustom(kind="custom", D=Dg), t, W, Xi, M, Dg)
    g = torch.empty_like(m.params)
    out = m._run(t.to(dev), W.to(dev), Xi.to(dev), grad=g, want=("X", "Y", "Z"))
    torch.cuda.synchronize()
    _compare(out, g, ref, ref["used"])
