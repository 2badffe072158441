"""The plugin API's host logic (generic.py) on the CPU: override detection
against a problem_spec, the Y/Z-dependence check, and the decomposition the
generic path rests on -- rollout first, the residual loss on detached (u, Z)
leaves, its cotangents contracted through (u, Z)'s VJP -- against the oracle's
autograd of the reference loss (nd_BSPDE_case.py:237-281).  The native
net_u / net_u_vjp are replaced by torch autograd of the oracle network here;
tests/test_gpu_plugin.py runs the real path.  Also the stream-order selection
of the C library (dbsde_stream_order_by_events) over synthetic environments."""
import ctypes
import importlib
import types

import numpy as np
import pytest
import torch

from conftest import load_pkg
from oracle import fbsnn_ref as fr

pkg = load_pkg()
gen = importlib.import_module(pkg.__name__ + ".generic")
fbm = importlib.import_module(pkg.__name__ + ".fbsnn")


class CustomProblem(fr.Problem):
    """A problem ProblemSpec cannot express: time-dependent drift, additive
    time-dependent diffusion, a |Z| driver and a quartic payoff."""

    def mu(self, t, X, Y, Z):
        return 0.05 * X * (1 + t)

    def sigma(self, t, X, Y):
        return torch.diag_embed(0.2 * X + 0.05 * t)

    def phi(self, t, X, Y, Z):
        return 0.05 * Y + 0.1 * torch.sqrt(torch.sum(Z ** 2, dim=1, keepdim=True))

    def g(self, X):
        return torch.sum(X ** 2, dim=1, keepdim=True) ** 2 / self.D


def fake_fb(problem, D):
    """An object with the reference's method surface over an oracle Problem."""
    ns = types.SimpleNamespace()
    ns.mu_tf = problem.mu
    ns.sigma_tf = problem.sigma
    ns.phi_tf = problem.phi
    ns.g_tf = problem.g

    def Dg_tf(X):
        X = X.detach().requires_grad_(True)
        v = problem.g(X)
        return torch.autograd.grad(v, X, torch.ones_like(v))[0]
    ns.Dg_tf = Dg_tf
    ns.state_dim = D
    return ns


@pytest.mark.parametrize("D,M,N", [(8, 16, 6), (1, 5, 4)])
def test_generic_decomposition_equals_autograd_double_backward(D, M, N):
    torch.manual_seed(3)
    np.random.seed(3)
    prob = CustomProblem(kind="custom", D=D)
    model = fr.build_model("Naisnet", [D + 1, 16, 16, 16, 1], "Sine")
    t, W = fr.fetch_minibatch(M, N, D, 1.0)
    Xi = torch.from_numpy(np.random.uniform(0.5, 1.5, (1, D))).float()
    ref = fr.loss_and_grads(model, prob, t, W, Xi, M, D)

    fb = fake_fb(prob, D)
    X, sdw = gen.rollout(fb, t, W, Xi.repeat(M, 1))
    np.testing.assert_array_equal(X.numpy(), ref["X"])          # the rollout is the reference's, op for op
    R = M * (N + 1)
    trow, xrow = t.reshape(R, 1), X.reshape(R, D).clone().requires_grad_(True)
    u, du = fr.net_u(model, trow, xrow)                            # stands in for dbsde_net_u
    U = u.detach().view(M, N + 1, 1).requires_grad_(True)
    DU = du.detach().view(M, N + 1, D).requires_grad_(True)
    loss = gen.residual_loss(fb, t, X, U, DU, sdw)
    assert float(loss) == pytest.approx(ref["loss"], rel=1e-5)
    ub, zb = torch.autograd.grad(loss, (U, DU))
    model.zero_grad(set_to_none=True)
    torch.autograd.backward((u, du), (ub.reshape(R, 1), zb.reshape(R, D)))   # stands in for dbsde_net_u_vjp
    g, _ = fr.flat_grads(model)
    np.testing.assert_allclose(g, ref["grad"], rtol=0, atol=1e-5 * np.abs(ref["grad"]).max())


class _Base:
    """Stands in for fbsnn.FBSNN (the override detection walks the MRO)."""

    def mu_tf(self, t, X, Y, Z):
        return torch.zeros_like(X)

    def sigma_tf(self, t, X, Y):
        return torch.diag_embed(torch.ones_like(X))

    def phi_tf(self, t, X, Y, Z):
        raise NotImplementedError

    def g_tf(self, X):
        raise NotImplementedError

    def Dg_tf(self, X):
        X = X.detach().requires_grad_(True)
        v = self.g_tf(X)
        return torch.autograd.grad(v, X, torch.ones_like(v))[0]


class _BSB(_Base):
    strike = 0.0

    def phi_tf(self, t, X, Y, Z):
        return 0.05 * (Y - torch.sum(X * Z, dim=1, keepdim=True))

    def g_tf(self, X):
        return torch.sum(X ** 2, 1, keepdim=True)

    def sigma_tf(self, t, X, Y):
        return 0.4 * torch.diag_embed(X)


class _MyBSB(_BSB):
    def sigma_tf(self, t, X, Y):
        return 0.3 * torch.diag_embed(X)


BSB_SPEC = pkg.ProblemSpec(sig_a=0.4, phi_r=0.05, phi_c=1.0, g="sumsq")


def test_override_detection():
    xi = torch.ones(1, 6)
    assert gen.coefficient_mismatches(_BSB(), _Base, BSB_SPEC, 6, 1.0, xi, "cpu") == []
    assert gen.coefficient_mismatches(_MyBSB(), _Base, BSB_SPEC, 6, 1.0, xi, "cpu") == ["sigma_tf"]

    class Drift(_BSB):
        def mu_tf(self, t, X, Y, Z):
            return 0.01 * X * t

    class Payoff(_BSB):
        def g_tf(self, X):
            return torch.sum(X ** 2, 1, keepdim=True) + 1.0

    class SameAgain(_BSB):               # an override that restates the spec is not a mismatch
        def phi_tf(self, t, X, Y, Z):
            return 0.05 * Y - 0.05 * torch.sum(X * Z, dim=1, keepdim=True)

    class Shape(_BSB):                   # a method that cannot be evaluated on the probes
        def mu_tf(self, t, X, Y, Z):
            return torch.zeros(3, 2)

    assert gen.coefficient_mismatches(Drift(), _Base, BSB_SPEC, 6, 1.0, xi, "cpu") == ["mu_tf"]
    assert gen.coefficient_mismatches(Payoff(), _Base, BSB_SPEC, 6, 1.0, xi, "cpu") == ["g_tf"]
    assert gen.coefficient_mismatches(SameAgain(), _Base, BSB_SPEC, 6, 1.0, xi, "cpu") == []
    assert gen.coefficient_mismatches(Shape(), _Base, BSB_SPEC, 6, 1.0, xi, "cpu") == ["mu_tf"]


def test_package_problem_methods_agree_with_their_specs():
    """Every shipped DIAG problem's torch methods equal its problem_spec on the
    probes (so none of them leaves the native path)."""
    base = fbm.FBSNN
    for cls, D, strike in ((pkg.CallOption, 5, 5.0), (pkg.CallOption1D, 1, 1.0), (pkg.BasketCallOption, 5, 1.0),
                           (pkg.BSPDETestCase, 5, 1.0), (pkg.HamiltonJacobiBellman, 5, 1.0),
                           (pkg.BlackScholesBarenblatt, 5, 0.0)):
        obj = object.__new__(cls)
        obj.strike, obj.D, obj.M, obj.device = strike, D, 4, torch.device("cpu")
        spec = cls.problem_spec(obj)
        assert gen.coefficient_mismatches(obj, base, spec, D, 1.0, torch.ones(1, D), "cpu") == [], cls.__name__

    class MyBSB(pkg.BlackScholesBarenblatt):
        def sigma_tf(self, t, X, Y):
            return 0.3 * torch.diag_embed(X)
    obj = object.__new__(MyBSB)
    obj.strike, obj.D, obj.device = 0.0, 5, torch.device("cpu")
    assert gen.coefficient_mismatches(obj, base, obj.problem_spec(), 5, 1.0, torch.ones(1, 5), "cpu") == ["sigma_tf"]


def test_spec_functions_match_oracle_problem_table():
    """generic.spec_functions (the override check's notion of a spec) against
    the oracle's restated coefficients of every DIAG problem."""
    torch.manual_seed(0)
    D = 4
    t, X, Y, Z = torch.rand(7, 1), 0.5 + torch.rand(7, D), torch.randn(7, 1), torch.randn(7, D)
    specs = {"bsb": (pkg.BlackScholesBarenblatt, 0.0), "call": (pkg.CallOption, 4.0),
             "basket": (pkg.BasketCallOption, 1.0), "bspde_test": (pkg.BSPDETestCase, 1.0),
             "hjb": (pkg.HamiltonJacobiBellman, 1.0)}
    for kind, (cls, strike) in specs.items():
        spec = cls.problem_spec(types.SimpleNamespace(strike=strike, D=D))
        f = gen.spec_functions(spec)
        p = fr.Problem(kind=kind, D=D, strike=strike)
        torch.testing.assert_close(f["mu_tf"](t, X, Y, Z), p.mu(t, X, Y, Z))
        torch.testing.assert_close(f["sigma_tf"](t, X, Y), p.sigma(t, X, Y))
        torch.testing.assert_close(f["phi_tf"](t, X, Y, Z), p.phi(t, X, Y, Z))
        torch.testing.assert_close(f["g_tf"](X), p.g(X))


def test_state_dependence_is_rejected():
    class YDrift(_BSB):
        def mu_tf(self, t, X, Y, Z):
            return 0.05 * X + 0.01 * Y

    class ZVol(_BSB):
        def sigma_tf(self, t, X, Y):
            return torch.diag_embed(0.2 * X * (1 + 0.0 * Y) + 0.01 * Y)

    class Harmless(_BSB):               # reads Y with a zero coefficient: X still independent
        def mu_tf(self, t, X, Y, Z):
            return 0.05 * X + 0.0 * Y

    for cls in (YDrift, ZVol):
        with pytest.raises(ValueError, match="depends on Y or Z"):
            gen.state_independence(cls(), 4, 1.0, torch.ones(1, 4), "cpu")
    gen.state_independence(Harmless(), 4, 1.0, torch.ones(1, 4), "cpu")
    gen.state_independence(_MyBSB(), 4, 1.0, torch.ones(1, 4), "cpu")


def _order(lib, env):
    if env is None:
        return lib.dbsde_stream_order_by_events(None)
    arr = (ctypes.c_char_p * (len(env) + 1))(*[e.encode() for e in env], None)
    return lib.dbsde_stream_order_by_events(arr)


def test_stream_order_selection_over_environments():
    """Value waits spin until the writer's queue runs the write, so any
    serialising or profiling environment must select event ordering
    (include/dbsde.h dbsde_stream_order_by_events).  Synthetic environments:
    the process environment is not touched."""
    importlib.import_module(pkg.__name__ + ".build_lib").build(verbose=False)
    lib = pkg._lib.load()
    assert _order(lib, []) == 0
    assert _order(lib, ["PATH=/usr/bin", "HOME=/root", "LD_PRELOAD=/usr/lib/libfoo.so"]) == 0
    events = ["DBSDE_STREAM_ORDER=events", "AMD_SERIALIZE_KERNEL=3", "HIP_LAUNCH_BLOCKING=1",
              "ROCPROF_COUNTER_COLLECTION=1", "ROCPROF_COUNTERS=SQ_WAVES", "HSA_TOOLS_LIB=/opt/rocm/lib/librocprofiler-sdk-tool.so",
              "LD_PRELOAD=/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so", "ROCPROFILER_OUTPUT_PATH=/tmp/x",
              "ROCP_TOOL_LIB=x.so"]
    for e in events:
        assert _order(lib, ["PATH=/usr/bin", e]) == 1, e
        if not e.startswith("DBSDE_"):
            assert _order(lib, [e, "DBSDE_STREAM_ORDER=values"]) == 0, e     # explicit override
    for e in ("AMD_SERIALIZE_KERNEL=0", "HIP_LAUNCH_BLOCKING=false", "HSA_TOOLS_LIB=", "ROCPROFX=1",
              "DBSDE_STREAM_ORDER=auto"):
        assert _order(lib, [e]) == 0, e
    assert _order(lib, None) in (0, 1)        # the process environment


def test_batched_residual_equals_the_per_step_loop():
    """generic.residual_loss over all M N rows at once (row-wise phi, D > 1)
    against the reference's per-step loop: the loss and its cotangents (u, Z)
    to fp32 summation-order rounding; a phi that couples the paths of a step
    is detected and keeps the loop."""
    torch.manual_seed(5)
    np.random.seed(5)
    D, M, N = 8, 12, 7
    prob = CustomProblem(kind="custom", D=D)
    fb = fake_fb(prob, D)
    assert gen.phi_row_independent(fb, D, "cpu")
    t, W = fr.fetch_minibatch(M, N, D, 1.0)
    Xi = torch.from_numpy(np.random.uniform(0.5, 1.5, (1, D))).float()
    X, sdw = gen.rollout(fb, t, W, Xi.repeat(M, 1))
    U = torch.randn(M, N + 1, 1, requires_grad=True)
    DU = torch.randn(M, N + 1, D, requires_grad=True)
    l0 = gen.residual_loss(fb, t, X, U, DU, sdw)
    l1 = gen.residual_loss(fb, t, X, U, DU, sdw, batched=True)
    assert float(l1) == pytest.approx(float(l0), rel=1e-6)
    g0 = torch.autograd.grad(l0, (U, DU))
    g1 = torch.autograd.grad(l1, (U, DU))
    for a, b in zip(g0, g1):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5 * float(a.abs().max()))

    coupled = fake_fb(prob, D)
    coupled.phi_tf = lambda t, X, Y, Z: 0.05 * Y + 0.1 * torch.sum(Z.mean(0, keepdim=True) * Z, dim=1, keepdim=True)
    assert not gen.phi_row_independent(coupled, D, "cpu")
    broken = fake_fb(prob, D)
    broken.phi_tf = lambda t, X, Y, Z: torch.sum(Y)   # not one value per row
    assert not gen.phi_row_independent(broken, D, "cpu")
