"""DeepBSDE.py surface: FBSNN(Xi, T, M, N, D, layers, mode, activation) with a
fixed N, no gradient clipping, train() returning only the loss graph and
loss_function() returning Y0 as a float (DeepBSDE.py:140-323), plus the
north-star problem BlackScholesBarenblatt (DeepBSDE.py:326-341) and its exact
solution u_exact (DeepBSDE.py:345-349)."""
from __future__ import annotations

import numpy as np
import torch

from . import fbsnn as _v2
from .solver import ProblemSpec


class FBSNN(_v2.FBSNN):
    clip_max_norm = None          # DeepBSDE.py:276-280 has no clip_grad_norm_
    schedule = None               # DeepBSDE.py has no N schedule

    def __init__(self, Xi, T, M, N, D, layers, mode, activation, device=None):
        super().__init__(Xi, T, M, N, D, None, layers, mode, activation, device=device)

    def loss_function(self, t, W, Xi):
        loss, X, Y, y0 = super().loss_function(t, W, Xi)
        return loss, X, Y, float(y0.item())

    def train(self, N_Iter, learning_rate):
        graph, _, _ = super().train(N_Iter, learning_rate, 'Adam')
        return graph

    def predict(self, Xi_star, t_star, W_star):
        return super().predict(Xi_star, t_star, W_star)


class BlackScholesBarenblatt(FBSNN):
    """DeepBSDE.py:326-341: mu = 0, sigma = 0.4 diag(X), phi = 0.05 (Y - X.Z), g = |X|^2."""

    def problem_spec(self):
        return ProblemSpec(sig_a=0.4, phi_r=0.05, phi_c=1.0, g="sumsq")

    def phi_tf(self, t, X, Y, Z):
        return 0.05 * (Y - torch.sum(X * Z, dim=1, keepdim=True))

    def g_tf(self, X):
        return torch.sum(X ** 2, 1, keepdim=True)

    def sigma_tf(self, t, X, Y):
        return 0.4 * torch.diag_embed(X)


def u_exact(t, X, T=1.0):
    """DeepBSDE.py:345-349: exp((r + sigma_max^2)(T - t)) |X|^2."""
    r, sigma_max = 0.05, 0.4
    return np.exp((r + sigma_max ** 2) * (T - t)) * np.sum(X ** 2, 1, keepdims=True)


__all__ = ["FBSNN", "BlackScholesBarenblatt", "u_exact"]
