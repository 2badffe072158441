"""Problem classes of the reference, as FBSNN subclasses with native
coefficients (problem_spec) plus the reference's torch expressions for
phi_tf / g_tf / mu_tf / sigma_tf.  The native step runs the spec; the methods
are compared with it on probe inputs at construction (fbsnn._select_problem),
so a subclass overriding one of them with other coefficients runs its own
methods (generic.py) instead of silently training the parent's problem.

  CallOption            nd_BSPDE_case.py:503-539        sum-payoff call, phi = r(Y - X.Z)
  CallOption1D          1d_BSPDE_case.py:510-560        1-D call, phi = 0.01 Y (Q3 broadcast)
  BasketCallOption      with_corr...py:546-596          mean-payoff basket, correlated dW
  BSPDETestCase         with_corr...py:599-616          sum X^2 payoff, mu = 0.05 X
  HamiltonJacobiBellman hjb_implement.py:590-604        phi = |Z|^2, g = log(1/2 + |X|^2/2)
  HestonFBSNN           heston_dnnpde.py:519-699        k-asset stochastic volatility
  BlackScholesBarenblatt: see deepbsde.py (DeepBSDE.py:326-341 surface)
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import networks
from .fbsnn import FBSNN
from .solver import ProblemSpec


class CallOption(FBSNN):
    """nd_BSPDE_case.py:503-539."""

    def problem_spec(self):
        return ProblemSpec(mu_a=0.05, sig_a=0.20, phi_r=0.05, phi_c=1.0, g="call_sum", strike=self.strike)

    def phi_tf(self, t, X, Y, Z):
        return 0.05 * (Y - torch.sum(X * Z, dim=1, keepdim=True))

    def g_tf(self, X):
        return torch.maximum(torch.sum(X, dim=1, keepdim=True) - self.strike, torch.tensor(0.0, device=X.device))

    def mu_tf(self, t, X, Y, Z):
        return 0.05 * X

    def sigma_tf(self, t, X, Y):
        return 0.20 * torch.diag_embed(X)


class CallOption1D(FBSNN):
    """1d_BSPDE_case.py:510-560 (strike = D; the D == 1 squeeze broadcast of
    1d_BSPDE_case.py:271-273 is reproduced)."""

    def problem_spec(self):
        return ProblemSpec(mu_a=0.01, sig_a=0.25, phi_r=0.01, phi_c=0.0, g="call_sum", strike=self.strike, q3=True)

    def phi_tf(self, t, X, Y, Z):
        return 0.01 * Y

    def g_tf(self, X):
        return torch.maximum(torch.sum(X, dim=1, keepdim=True) - self.strike, torch.tensor(0.0, device=X.device))

    def mu_tf(self, t, X, Y, Z):
        return 0.01 * X

    def sigma_tf(self, t, X, Y):
        return 0.25 * torch.diag_embed(X)


class _WithCorrTrain:
    """The train() surface of with_corr_high_dimension_pde.py:355-453: log and
    record every 500 iterations (no print), return (graph, min_loss,
    min_loss_state, time_logs)."""

    schedule = "corr"
    log_every = 500
    log_print = False
    train_returns_time_logs = True


class BasketCallOption(_WithCorrTrain, FBSNN):
    """with_corr_high_dimension_pde.py:546-596 (its FBSNN sets strike = 1.0 and
    applies the N**(1/5) schedule of with_corr...:406-409)."""

    def _default_strike(self):
        return 1.0

    def problem_spec(self):
        return ProblemSpec(mu_a=0.05, sig_a=0.20, phi_r=0.05, phi_c=0.0, g="call_mean", strike=self.strike)

    def phi_tf(self, t, X, Y, Z):
        return 0.05 * (Y)

    def g_tf(self, X):
        return torch.maximum(torch.mean(X, dim=1, keepdim=True) - self.strike, torch.tensor(0.0, device=X.device))

    def mu_tf(self, t, X, Y, Z):
        return 0.05 * X

    def sigma_tf(self, t, X, Y):
        return 0.20 * torch.diag_embed(X)


class BSPDETestCase(_WithCorrTrain, FBSNN):
    """with_corr_high_dimension_pde.py:599-616."""

    def _default_strike(self):
        return 1.0

    def problem_spec(self):
        return ProblemSpec(mu_a=0.05, sig_a=0.20, phi_r=0.05, phi_c=1.0, g="sumsq")

    def phi_tf(self, t, X, Y, Z):
        return 0.05 * (Y - torch.sum(X * Z, dim=1, keepdim=True))

    def g_tf(self, X):
        return torch.sum(X ** 2, dim=1, keepdim=True)

    def mu_tf(self, t, X, Y, Z):
        return 0.05 * X

    def sigma_tf(self, t, X, Y):
        return 0.20 * torch.diag_embed(X)


class HamiltonJacobiBellman(FBSNN):
    """hjb_implement.py:590-604.  The reference passes Mm=None and therefore
    cannot train (np.ceil(None)); here Mm=None means a fixed N.
    Its train() (hjb_implement.py:394-450) logs and prints every 500
    iterations and returns (graph, min_loss, min_loss_state, time_logs)."""

    log_every = 500
    train_returns_time_logs = True

    def __init__(self, Xi, T, M, N, D, layers, mode, activation, **kw):
        super().__init__(Xi, T, M, N, D, None, layers, mode, activation, **kw)

    def _default_strike(self):
        return 1.0

    def problem_spec(self):
        return ProblemSpec(sig_b=math.sqrt(2.0), phi_zz=1.0, g="log")

    def phi_tf(self, t, X, Y, Z):
        return torch.sum(Z ** 2, dim=1, keepdim=True)

    def g_tf(self, X):
        return torch.log(0.5 + 0.5 * torch.sum(X ** 2, dim=1, keepdim=True))

    def sigma_tf(self, t, X, Y):
        return math.sqrt(2.0) * super().sigma_tf(t, X, Y)


class HestonFBSNN(FBSNN):
    """heston_dnnpde.py:519-699, generalised from one asset to k = D assets.

    State [S_1..S_k, v_1..v_k] (k = 1 is the reference's [S, v]); one Brownian
    motion per asset drives both S_i and v_i (the reference's FBSNN dimension is
    1 and its einsum broadcasts dW, :522, :638); mu and the 2x2 diffusion block
    of each asset are clamped to [-100, 100] (:591, :605); u = max(net, 0)
    (:568); phi = 0.05 Y; the terminal payoff is the call on mean S (the
    reference's max(S - 1, 0) at k = 1, or its sigmoid-smoothed "continuous"
    variant, :546-558) and the terminal Z term uses dU/dS only (:654).  The
    network takes (t, S, v) -- 1 + 2k inputs -- and is initialised as the
    reference re-initialises it (xavier gain 0.5, zero biases, :580-585).
    An iteration whose loss is NaN is skipped (:409-411).  k > 1 has no
    reference golden; k = 1 is pinned by tests/golden/g1_heston_*."""

    skip_nonfinite = True
    log_print = False             # its progress print is commented out (heston_dnnpde.py:432-434)

    def __init__(self, Xi, T, M, N, D, Mm, layers, mode, activation, correlation_type="no_correlation",
                 kappa=2.0, theta=0.2, sigma=0.3, rho=0.8, v0=0.2, payoff_type='discontinuous', device=None):
        if payoff_type not in ("discontinuous", "continuous"):
            raise ValueError("Invalid payoff type. Choose 'discontinuous' or 'continuous'.")
        self.kappa, self.theta, self.sigma, self.rho, self.v0 = kappa, theta, sigma, rho, v0
        self.payoff_type = payoff_type
        self.n_assets = D
        self.Y0_values = []
        self.y0_values = []
        super().__init__(Xi, T, M, N, D, Mm, layers, mode, activation, correlation_type, device=device)

    def _default_strike(self):
        return 1.0

    def _native_layers(self, layers):
        return [1 + 2 * self.n_assets] + layers[1:]

    def _make_model(self, layers):
        return networks.make_heston_model(self.mode, layers, self.activation, 1 + 2 * self.n_assets)

    def _full_state(self, Xi):
        """[S_1..S_k, ...] -> [S_1..S_k, v0..v0]: the reference always starts the
        variance at self.v0 and reads only the S column(s) of Xi
        (heston_dnnpde.py:619-623; predict may append v0, :668-670, which
        loss_function then ignores)."""
        k = self.n_assets
        x = torch.as_tensor(np.asarray(Xi) if not isinstance(Xi, torch.Tensor) else Xi,
                            dtype=torch.float32).to(self.device)
        x = x.reshape(-1, x.shape[-1]) if x.dim() > 1 else x.reshape(1, -1)
        if x.shape[1] < k:
            raise ValueError(f"Xi has {x.shape[1]} columns; the {k} asset prices come first")
        S = x[:, :k]
        return torch.cat([S, torch.full_like(S, self.v0)], 1).contiguous()

    def _initial_state(self, Xi):
        return self._full_state(Xi)

    def problem_spec(self):
        smooth = self.payoff_type == "continuous"
        return ProblemSpec(kind="heston", mu_a=0.05, phi_r=0.05, phi_c=0.0, g="smooth_call" if smooth else "call_mean",
                           strike=self.strike, g_alpha=10.0, g_cols=self.n_assets, u_clamp=True, q3=False,
                           kappa=self.kappa, theta=self.theta, sigma=self.sigma, rho=self.rho)

    def g_tf(self, X):
        S = X[:, :self.n_assets] if X.dim() > 1 else X
        a = torch.mean(S, dim=1, keepdim=True) - self.strike if S.dim() > 1 else S - self.strike
        if self.payoff_type == "discontinuous":
            return torch.maximum(a, torch.tensor(0.0, device=X.device))
        return a / (1 + torch.exp(-10.0 * a))

    def phi_tf(self, t, X, Y, Z):
        return 0.05 * Y

    def mu_tf(self, t, X, Y=None, Z=None):
        k = self.n_assets
        S, v = X[:, :k], X[:, k:]
        return torch.cat([0.05 * S, self.kappa * (self.theta - v)], dim=1).clamp(-100, 100)

    def _record_y0(self, out):
        y0 = float(out["Y"][0, 0, 0])
        self.Y0_values.append(y0)

    def _train_graph(self):
        return np.column_stack((self.iteration, self.training_loss, self.Y0_values))

    def train(self, N_Iter, learning_rate, optimizer_type='Adam'):
        """heston_dnnpde.py:345-450 -> graph [iteration, training_loss, Y0]."""
        graph, _, _ = super().train(N_Iter, learning_rate, optimizer_type)
        return graph

    def predict(self, Xi_star, t_star, W_star):
        """heston_dnnpde.py:661-683 -> (S, v, Y)."""
        X, Y = super().predict(self._full_state(Xi_star), t_star, W_star)
        k = self.n_assets
        return X[:, :, :k], X[:, :, k:], Y


__all__ = ["CallOption", "CallOption1D", "BasketCallOption", "BSPDETestCase", "HamiltonJacobiBellman",
           "HestonFBSNN"]
