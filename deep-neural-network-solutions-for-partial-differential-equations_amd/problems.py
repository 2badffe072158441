"""Problem classes of the reference, as FBSNN subclasses with native
coefficients (problem_spec) plus the reference's torch expressions for
phi_tf / g_tf / mu_tf / sigma_tf (API completeness; the native path does not
call them).

  CallOption            nd_BSPDE_case.py:503-539        sum-payoff call, phi = r(Y - X.Z)
  CallOption1D          1d_BSPDE_case.py:510-560        1-D call, phi = 0.01 Y (Q3 broadcast)
  BasketCallOption      with_corr...py:546-596          mean-payoff basket, correlated dW
  BSPDETestCase         with_corr...py:599-616          sum X^2 payoff, mu = 0.05 X
  HamiltonJacobiBellman hjb_implement.py:590-604        phi = |Z|^2, g = log(1/2 + |X|^2/2)
  BlackScholesBarenblatt: see deepbsde.py (DeepBSDE.py:326-341 surface)
"""
from __future__ import annotations

import math

import torch

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


class BasketCallOption(FBSNN):
    """with_corr_high_dimension_pde.py:546-596 (its FBSNN sets strike = 1.0 and
    applies the N**(1/5) schedule of with_corr...:406-409)."""

    schedule = "corr"

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


class BSPDETestCase(FBSNN):
    """with_corr_high_dimension_pde.py:599-616."""

    schedule = "corr"

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
    cannot train (np.ceil(None)); here Mm=None means a fixed N."""

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


__all__ = ["CallOption", "CallOption1D", "BasketCallOption", "BSPDETestCase", "HamiltonJacobiBellman"]
