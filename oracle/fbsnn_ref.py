"""ORACLE -- test infrastructure only, never the product path.

CPU restatement (torch, autograd) of the reference deep-BSDE training step, op
for op in the reference's order, so that it can act as the checker for the
HIP path and as the `cpu_baseline` ("port") leg of bench.py.  Only `tests/`,
`__graft_entry__.smoke()` and bench.py's cpu_baseline leg may import it.

Pinned against golden vectors produced by importing the reference itself in
the build container (tests/golden/make_golden.py -> tests/golden/*.npz,
checked by tests/test_oracle_golden.py).

What it restates (file:line into the reference snapshot):
  networks     DeepBSDE.py:23-65 / Functions/networks.py:8-50 (Resnet, stable
               = "NAIS-Net"), Functions/naisnet.py:6-96 / nd_BSPDE_case.py:33-123
               (Naisnet, fixed depth), DeepBSDE.py:166-172 (FC nn.Sequential),
               Functions/Sine.py:6-12 (Sine), DeepBSDE.py:185-187 (xavier init)
  net_u        DeepBSDE.py:189-194, nd_BSPDE_case.py:191-221
  Dg_tf        DeepBSDE.py:196-200
  loss         DeepBSDE.py:202-245, nd_BSPDE_case.py:237-281 (+ the D=1
               squeeze broadcast of 1d_BSPDE_case.py:271-273)
  minibatch    DeepBSDE.py:247-262, with_corr_high_dimension_pde.py:316-353
  problems     DeepBSDE.py:326-341 (BSB), nd_BSPDE_case.py:503-539 (CallOption),
               1d_BSPDE_case.py:510-560 (1-D call), with_corr...:546-596
               (basket CallOption), with_corr...:599-616 (BSPDETestCase),
               hjb_implement.py:590-604 (HJB), heston_dnnpde.py:519-659 (Heston:
               own net_u with the u clamp, own loss_function, k = 1 exactly as
               the reference; k > 1 the per-asset generalisation)
  train step   nd_BSPDE_case.py:316-410 (N schedule, clip 1.0, Adam),
               DeepBSDE.py:265-295 (no schedule, no clip)
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# --------------------------------------------------------------------------
# networks
# --------------------------------------------------------------------------


class SineAct(nn.Module):
    """Functions/Sine.py:6-12."""

    def forward(self, x):
        return torch.sin(x)


def make_activation(name: str) -> nn.Module:
    if name == "Sine":
        return SineAct()
    if name == "ReLU":
        return nn.ReLU()
    if name == "Tanh":
        return nn.Tanh()
    raise ValueError(f"unknown activation {name!r}")


def _projected(weight: torch.Tensor, eps: float = 0.01) -> torch.Tensor:
    """NAIS-Net stability projection, Functions/naisnet.py:30-39.

    Returns A (not -A).  The data-dependent branch is a Python branch on the
    Frobenius norm, exactly as the reference takes it.
    """
    delta = 1 - 2 * eps
    rtr = torch.matmul(weight.t(), weight)
    nrm = torch.norm(rtr)
    if nrm > delta:
        rtr = delta ** (1 / 2) * rtr / (nrm ** (1 / 2))
    return rtr + torch.eye(rtr.shape[0], dtype=rtr.dtype, device=rtr.device) * eps


class ResnetRef(nn.Module):
    """DeepBSDE.py:23-65.  stable=True is the "NAIS-Net" mode.

    Registration order (input_layer, hidden_layers, output_layer,
    input_layers) fixes both the state_dict order and the RNG stream of the
    default nn.Linear init.  The last entry of input_layers is never used by
    forward.
    """

    def __init__(self, layers, stable, act):
        super().__init__()
        self.stable = stable
        self.epsilon = 0.01
        self.act = act
        self.input_layer = nn.Linear(layers[0], layers[1])
        self.hidden_layers = nn.ModuleList(
            [nn.Linear(layers[i], layers[i + 1]) for i in range(1, len(layers) - 2)])
        self.output_layer = nn.Linear(layers[-2], layers[-1])
        if stable:
            self.input_layers = nn.ModuleList(
                [nn.Linear(layers[0], layers[i]) for i in range(1, len(layers) - 1)])

    def forward(self, x):
        h = self.act(self.input_layer(x))
        for k, lin in enumerate(self.hidden_layers):
            res = h.clone()
            if self.stable:
                a = F.linear(h, -_projected(lin.weight, self.epsilon), lin.bias)
                a = a + self.input_layers[k](x)
            else:
                a = lin(h)
            h = self.act(a) + res
        return self.output_layer(h)


class NaisnetRef(nn.Module):
    """Functions/naisnet.py:6-96 == nd_BSPDE_case.py:33-123 (len(layers) 4/5/6).

    Same algebra as ResnetRef(stable=True) but with the layerN/layerN_input
    naming of the reference and no unused parameters.  The reference builds
    eye() on the CPU; the restatement builds it on the weight's
    device, which is the only behaviour the reference can have on CPU.
    """

    def __init__(self, layers, act):
        super().__init__()
        n = len(layers)
        if n not in (4, 5, 6):
            raise ValueError("Naisnet supports len(layers) in {4,5,6}")
        self.nl = n
        self.act = act
        self.epsilon = 0.01
        self.layer1 = nn.Linear(layers[0], layers[1])
        self.layer2 = nn.Linear(layers[1], layers[2])
        self.layer2_input = nn.Linear(layers[0], layers[2])
        self.layer3 = nn.Linear(layers[2], layers[3])
        if n >= 5:
            self.layer3_input = nn.Linear(layers[0], layers[3])
            self.layer4 = nn.Linear(layers[3], layers[4])
        if n == 6:
            self.layer4_input = nn.Linear(layers[0], layers[4])
            self.layer5 = nn.Linear(layers[4], layers[5])

    def _block(self, lin, inj, h, x):
        a = F.linear(h, -_projected(lin.weight, self.epsilon), lin.bias) + inj(x)
        return self.act(a) + h

    def forward(self, x):
        h = self.act(self.layer1(x))
        h = self._block(self.layer2, self.layer2_input, h, x)
        if self.nl == 4:
            return self.layer3(h)
        h = self._block(self.layer3, self.layer3_input, h, x)
        if self.nl == 5:
            return self.layer4(h)
        h = self._block(self.layer4, self.layer4_input, h, x)
        return self.layer5(h)


def build_model(mode: str, layers, activation: str) -> nn.Module:
    """Mirror of the mode switch in DeepBSDE.py:166-178 / nd_BSPDE_case.py:159-172,
    followed by model.apply(weights_init) (DeepBSDE.py:180,185-187)."""
    act = make_activation(activation)
    if mode == "FC":
        mods = []
        for i in range(len(layers) - 2):
            mods.append(nn.Linear(layers[i], layers[i + 1]))
            mods.append(act)
        mods.append(nn.Linear(layers[-2], layers[-1]))
        model = nn.Sequential(*mods)
    elif mode in ("NAIS-Net", "Resnet"):
        model = ResnetRef(layers, stable=(mode == "NAIS-Net"), act=act)
    elif mode == "Naisnet":
        model = NaisnetRef(layers, act)
    else:
        raise ValueError(f"unsupported mode {mode!r}")

    def _init(m):
        if isinstance(m, nn.Linear):
            torch.nn.init.xavier_uniform_(m.weight)

    model.apply(_init)
    return model


def flat_params(model) -> np.ndarray:
    return torch.cat([p.detach().reshape(-1) for p in model.state_dict().values()]).cpu().numpy()


def set_flat_params(model, flat) -> None:
    flat = torch.as_tensor(np.asarray(flat))
    off = 0
    with torch.no_grad():
        for p in model.state_dict().values():
            n = p.numel()
            p.copy_(flat[off:off + n].reshape(p.shape).to(p.dtype))
            off += n
    assert off == flat.numel()


def flat_grads(model):
    """(grad vector, used mask); params whose .grad is None (Q6) give zeros/False."""
    gs, mask = [], []
    params = dict(model.named_parameters())
    for name, p in model.state_dict().items():
        q = params[name]
        if q.grad is None:
            gs.append(torch.zeros(q.numel(), dtype=q.dtype))
            mask.append(np.zeros(q.numel(), dtype=bool))
        else:
            gs.append(q.grad.detach().reshape(-1).cpu())
            mask.append(np.ones(q.numel(), dtype=bool))
    return torch.cat(gs).numpy(), np.concatenate(mask)


# --------------------------------------------------------------------------
# problems
# --------------------------------------------------------------------------


@dataclass
class Problem:
    """Problem coefficients.  Each expression is the reference's own, in its
    own operation order (file:line in the module docstring)."""

    kind: str
    D: int
    strike: float = 0.0
    q3_compat: bool = False      # 1d_BSPDE_case.py squeeze broadcast (Q3)
    extra: dict = field(default_factory=dict)

    def mu(self, t, X, Y, Z):
        k = self.kind
        if k in ("bsb", "hjb"):
            return torch.zeros([X.shape[0], self.D], dtype=X.dtype)
        if k in ("call", "basket", "bspde_test"):
            return 0.05 * X
        if k == "call1d":
            return 0.01 * X
        raise ValueError(k)

    def sigma(self, t, X, Y):
        k = self.kind
        if k == "bsb":
            return 0.4 * torch.diag_embed(X)
        if k in ("call", "basket", "bspde_test"):
            return 0.20 * torch.diag_embed(X)
        if k == "call1d":
            return 0.25 * torch.diag_embed(X)
        if k == "hjb":
            return torch.sqrt(torch.tensor(2.0)) * torch.diag_embed(
                torch.ones([X.shape[0], self.D], dtype=X.dtype))
        raise ValueError(k)

    def phi(self, t, X, Y, Z):
        k = self.kind
        if k in ("bsb", "call", "bspde_test"):
            return 0.05 * (Y - torch.sum(X * Z, dim=1, keepdim=True))
        if k == "basket":
            return 0.05 * (Y)
        if k == "call1d":
            return 0.01 * (Y)
        if k == "hjb":
            return torch.sum(Z ** 2, dim=1, keepdim=True)
        raise ValueError(k)

    def g(self, X):
        k = self.kind
        if k in ("bsb", "bspde_test"):
            return torch.sum(X ** 2, 1, keepdim=True)
        if k in ("call", "call1d"):
            return torch.maximum(torch.sum(X, dim=1, keepdim=True) - self.strike,
                                 torch.tensor(0.0, dtype=X.dtype))
        if k == "basket":
            return torch.maximum(torch.mean(X, dim=1, keepdim=True) - self.strike,
                                 torch.tensor(0.0, dtype=X.dtype))
        if k == "hjb":
            return torch.log(0.5 + 0.5 * torch.sum(X ** 2, dim=1, keepdim=True))
        raise ValueError(k)


def make_problem(kind: str, D: int) -> Problem:
    """Strikes: nd/1d use strike = 1.0*D (nd_BSPDE_case.py:147, 1d:160);
    with_corr/hjb use 1.0 (with_corr...:153)."""
    strike = {"call": 1.0 * D, "call1d": 1.0 * D, "basket": 1.0}.get(kind, 0.0)
    return Problem(kind=kind, D=D, strike=strike, q3_compat=(kind == "call1d"))


# --------------------------------------------------------------------------
# solver core
# --------------------------------------------------------------------------


def fetch_minibatch(M, N, D, T, L=None, rng=None, dtype=torch.float32):
    """DeepBSDE.py:247-262; correlated increments with_corr...:339-341.

    Uses the legacy global numpy stream unless `rng` (a RandomState) is given.
    t and W are built in float64 and cast."""
    normal = (rng or np.random).normal
    Dt = np.zeros((M, N + 1, 1))
    DW = np.zeros((M, N + 1, D))
    dt = T / N
    Dt[:, 1:, :] = dt
    dwu = np.sqrt(dt) * normal(size=(M, N, D))
    DW[:, 1:, :] = dwu if L is None else np.einsum('ij,mnj->mni', L, dwu)
    t = np.cumsum(Dt, axis=1)
    W = np.cumsum(DW, axis=1)
    return torch.from_numpy(t).to(dtype), torch.from_numpy(W).to(dtype)


def net_u(model, t, X):
    """DeepBSDE.py:189-194: u and Du = du/dX with create_graph."""
    inp = torch.cat((t, X), 1)
    u = model(inp)
    du = torch.autograd.grad(outputs=u, inputs=X, grad_outputs=torch.ones_like(u),
                             allow_unused=True, retain_graph=True, create_graph=True)[0]
    return u, du


def dg(problem, X):
    """DeepBSDE.py:196-200."""
    g = problem.g(X)
    return torch.autograd.grad(outputs=g, inputs=X, grad_outputs=torch.ones_like(g),
                               allow_unused=True, retain_graph=True, create_graph=True)[0]


def _squeeze_sdw(problem, sdw3):
    # nd/DeepBSDE squeeze(dim=-1) for X; the Y-tilde term uses squeeze() with
    # no dim (nd_BSPDE_case.py:263-265), which only differs from squeeze(-1)
    # when D == 1 (Q3).  Restated as the reference writes it.
    return torch.squeeze(sdw3)


def loss_function(model, problem, t, W, Xi, M, D):
    """nd_BSPDE_case.py:237-281 / DeepBSDE.py:202-245.

    Returns (loss, X[M,N+1,D], Y[M,N+1,1], Y0 float, Z[M,N+1,D])."""
    N = t.shape[1] - 1
    t0 = t[:, 0, :]
    W0 = W[:, 0, :]
    if Xi.shape[0] == 1:
        X0 = Xi.view(1, D).repeat(M, 1)
    else:
        X0 = Xi.view(M, D)
    Y0, Z0 = net_u(model, t0, X0)
    Xs, Ys, Zs = [X0], [Y0], [Z0]
    loss = 0
    for n in range(N):
        t1 = t[:, n + 1, :]
        W1 = W[:, n + 1, :]
        X1 = X0 + problem.mu(t0, X0, Y0, Z0) * (t1 - t0) + torch.squeeze(
            torch.matmul(problem.sigma(t0, X0, Y0), (W1 - W0).unsqueeze(-1)), dim=-1)
        Y1t = Y0 + problem.phi(t0, X0, Y0, Z0) * (t1 - t0) + torch.sum(
            Z0 * _squeeze_sdw(problem, torch.matmul(problem.sigma(t0, X0, Y0),
                                                    (W1 - W0).unsqueeze(-1))),
            dim=1, keepdim=True)
        Y1, Z1 = net_u(model, t1, X1)
        loss = loss + torch.sum(torch.pow(Y1 - Y1t, 2))
        t0, W0, X0, Y0, Z0 = t1, W1, X1, Y1, Z1
        Xs.append(X0)
        Ys.append(Y0)
        Zs.append(Z0)
    loss = loss + torch.sum(torch.pow(Y1 - problem.g(X1), 2))
    loss = loss + torch.sum(torch.pow(Z1 - dg(problem, X1), 2))
    X = torch.stack(Xs, dim=1)
    Y = torch.stack(Ys, dim=1)
    Z = torch.stack(Zs, dim=1)
    return loss, X, Y, float(Y[0, 0, 0].detach()), Z


def n_schedule(it: int, Mm: float, N: int) -> int:
    """nd_BSPDE_case.py:364-368: returns N for iteration `it`."""
    if 4000 <= it < 20000:
        return int(np.ceil(Mm ** (int(it / 4000) + 1)))
    if it < 4000:
        return int(np.ceil(Mm))
    return N


def loss_and_grads(model, problem, t, W, Xi, M, D):
    """One forward + autograd double backward; returns numpy results."""
    model.zero_grad(set_to_none=True)
    Xi = Xi.clone().requires_grad_(True)
    loss, X, Y, y0, Z = loss_function(model, problem, t, W, Xi, M, D)
    loss.backward()
    g, mask = flat_grads(model)
    return dict(loss=float(loss), X=X.detach().numpy(), Y=Y.detach().numpy(),
                Z=Z.detach().numpy(), Y0=y0, grad=g, used=mask)


def train(model, problem, Xi, M, N, D, T, n_iter, lr, clip=True, Mm=None,
          start_it=0, L=None, rng=None, schedule="nd", optimizer="Adam"):
    """nd_BSPDE_case.py:316-410 (clip=True, Mm schedule) or DeepBSDE.py:265-295
    (clip=False, Mm=None); schedule="corr" is with_corr...py:405-409 (N**(1/5)
    re-applied to the mutated N).  A fresh optimizer per call (Q11);
    optimizer="LBFGS" runs optimizer.step(closure) on the same batch without
    clipping (nd_BSPDE_case.py:357-361,380-381).  Returns per-iteration
    (loss, Y0) lists."""
    if optimizer == "LBFGS":
        opt = torch.optim.LBFGS(model.parameters(), lr=lr)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=lr)
    Xi_t = torch.as_tensor(Xi, dtype=torch.float32)
    losses, y0s = [], []
    for it in range(start_it, start_it + n_iter):
        if schedule == "corr":
            if 4000 <= it < 20000:
                N = int(np.ceil((N ** (1 / 5)) ** (int(it / 4000) + 1)))
            elif it < 4000:
                N = int(np.ceil(N ** (1 / 5)))
        elif Mm is not None:
            N = n_schedule(it, Mm, N)
        opt.zero_grad()
        t, W = fetch_minibatch(M, N, D, T, L=L, rng=rng)
        xi = Xi_t.clone().requires_grad_(True)
        loss, X, Y, y0, _ = loss_function(model, problem, t, W, xi, M, D)
        loss.backward()
        if optimizer == "LBFGS":
            def closure():
                opt.zero_grad()
                l2 = loss_function(model, problem, t, W, Xi_t.clone().requires_grad_(True), M, D)[0]
                l2.backward()
                return l2
            opt.step(closure)
        else:
            if clip:
                torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
            opt.step()
        losses.append(float(loss))
        y0s.append(y0)
    return losses, y0s


# --------------------------------------------------------------------------
# Heston (heston_dnnpde.py:519-659)
# --------------------------------------------------------------------------


def build_heston_model(mode, layers, activation, n_assets=1):
    """heston_dnnpde.py:522-585: base FBSNN model on `layers` (input D+1,
    default + xavier init), input-facing Linears replaced by (1 + 2k)-input
    ones, then every parameter re-initialised (xavier gain 0.5 / zeros)."""
    model = build_model(mode, layers, activation)
    n_in = 1 + 2 * n_assets
    if mode == "FC":
        model[0] = nn.Linear(n_in, layers[1])
    elif mode == "Naisnet":
        model.layer1 = nn.Linear(n_in, layers[1])
        model.layer2_input = nn.Linear(n_in, layers[2])
        if len(layers) >= 5:
            model.layer3_input = nn.Linear(n_in, layers[3])
        if len(layers) == 6:
            model.layer4_input = nn.Linear(n_in, layers[4])
    else:
        raise ValueError(mode)
    for prm in model.parameters():
        if len(prm.shape) > 1:
            torch.nn.init.xavier_uniform_(prm, gain=0.5)
        else:
            torch.nn.init.zeros_(prm)
    return model


@dataclass
class Heston:
    k: int = 1
    kappa: float = 2.0
    theta: float = 0.2
    sigma: float = 0.3
    rho: float = 0.8
    v0: float = 0.2
    payoff: str = "discontinuous"
    strike: float = 1.0

    def g(self, S):
        a = torch.mean(S, dim=1, keepdim=True) - self.strike if self.k > 1 else S - self.strike
        if self.payoff == "discontinuous":
            return torch.maximum(a, torch.tensor(0.0))
        return a / (1 + torch.exp(-10.0 * a))


def heston_net_u(model, t, X):
    """heston_dnnpde.py:560-579: u = clamp(model(t, S, v), min 0), Du over (S, v)."""
    u = model(torch.cat((t, X), 1))
    u = torch.clamp(u, min=0.0)
    du = torch.autograd.grad(outputs=u, inputs=X, grad_outputs=torch.ones_like(u), create_graph=True,
                             retain_graph=True)[0]
    return u, du


def heston_loss_function(model, h, t, W, Xi, M):
    """heston_dnnpde.py:611-659 per asset: X = [S_1..S_k, v_1..v_k], W [M, N+1, k].
    For k = 1 every expression is the reference's, in its order."""
    k = h.k
    N = t.shape[1] - 1
    t0, W0 = t[:, 0, :], W[:, 0, :]
    Xi = Xi.reshape(-1, Xi.shape[-1])
    S0 = Xi[:, :k].repeat(M, 1) if Xi.shape[0] == 1 else Xi[:, :k]
    v0 = torch.full((M, k), h.v0)
    X0 = torch.cat([S0, v0], dim=1)
    Y0, Z0 = heston_net_u(model, t0, X0)
    Xs, Ys, Zs = [X0], [Y0], [Z0]
    loss = 0
    for n in range(N):
        t1, W1 = t[:, n + 1, :], W[:, n + 1, :]
        dW = W1 - W0
        S, v = X0[:, :k], X0[:, k:]
        mu = torch.cat([0.05 * S, h.kappa * (h.theta - v)], dim=1).clamp(-100, 100)
        sv = torch.sqrt(torch.clamp(v, min=1e-8))
        sS, sV = sv * S, h.sigma * sv
        d00, d11 = sS.clamp(-100, 100), sV.clamp(-100, 100)
        d01, d10 = (h.rho * sV).clamp(-100, 100), (h.rho * sS).clamp(-100, 100)
        X1 = X0 + mu * (t1 - t0) + torch.cat([(d00 + d01) * dW, (d10 + d11) * dW], dim=1)
        a = d00 * dW + d01 * dW
        b = d10 * dW + d11 * dW
        Y1t = Y0 + 0.05 * Y0 * (t1 - t0) + torch.sum(Z0[:, :k] * a + Z0[:, k:] * b, dim=1, keepdim=True)
        Y1, Z1 = heston_net_u(model, t1, X1)
        loss = loss + torch.sum(torch.pow(Y1 - Y1t, 2))
        t0, W0, X0, Y0, Z0 = t1, W1, X1, Y1, Z1
        Xs.append(X0)
        Ys.append(Y0)
        Zs.append(Z0)
    loss = loss + torch.sum(torch.pow(Y1 - h.g(X1[:, :k]), 2))
    S1 = X1[:, :k]
    g = h.g(S1)
    dg = torch.autograd.grad(outputs=[g], inputs=[S1], grad_outputs=torch.ones_like(g), allow_unused=True,
                             retain_graph=True, create_graph=True)[0]
    loss = loss + torch.sum(torch.pow(Z1[:, :k] - dg, 2))
    return loss, torch.stack(Xs, 1), torch.stack(Ys, 1), torch.stack(Zs, 1)


def heston_loss_and_grads(model, h, t, W, Xi, M):
    model.zero_grad(set_to_none=True)
    xi = torch.as_tensor(Xi, dtype=torch.float32).clone().requires_grad_(True)   # the reference's Xi (:135)
    loss, X, Y, Z = heston_loss_function(model, h, t, W, xi, M)
    loss.backward()
    g, mask = flat_grads(model)
    return dict(loss=float(loss), X=X.detach().numpy(), Y=Y.detach().numpy(), Z=Z.detach().numpy(),
                grad=g, used=mask)


def heston_train(model, h, Xi, M, N, T, n_iter, lr, Mm=None, start_it=0):
    """heston_dnnpde.py:345-450: N schedule, Adam, NaN skip, clip 1.0; the
    minibatch has one Brownian column per asset (:309-343 with D = k)."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    losses = []
    for it in range(start_it, start_it + n_iter):
        if Mm is not None:
            N = n_schedule(it, Mm, N)
        opt.zero_grad()
        t, W = fetch_minibatch(M, N, h.k, T)
        xi = torch.as_tensor(Xi, dtype=torch.float32).clone().requires_grad_(True)
        loss, X, Y, Z = heston_loss_function(model, h, t, W, xi, M)
        if torch.isnan(loss):
            continue
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        losses.append(float(loss))
    return losses


def bsb_u_exact(t, X, T=1.0):
    """DeepBSDE.py:345-349 (the north-star known answer)."""
    r, smax = 0.05, 0.4
    return np.exp((r + smax ** 2) * (T - t)) * np.sum(X ** 2, 1, keepdims=True)


def param_count(mode, layers):
    return sum(int(np.prod(p.shape)) for p in build_model(mode, layers, "Sine").state_dict().values())


__all__ = [
    "SineAct", "ResnetRef", "NaisnetRef", "build_model", "flat_params", "set_flat_params",
    "flat_grads", "Problem", "make_problem", "fetch_minibatch", "net_u", "dg",
    "loss_function", "n_schedule", "loss_and_grads", "train", "bsb_u_exact", "param_count",
    "build_heston_model", "Heston", "heston_net_u", "heston_loss_function", "heston_loss_and_grads",
    "heston_train",
]

