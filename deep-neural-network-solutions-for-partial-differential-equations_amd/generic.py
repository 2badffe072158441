"""The reference's plugin API for problems the native coefficient table
(ProblemSpec) cannot express.

In the reference a problem is an FBSNN subclass overriding the abstract
phi_tf / g_tf / mu_tf / sigma_tf (nd_BSPDE_case.py:458-500; examples
CallOption nd_BSPDE_case.py:503-540, BlackScholesBarenblatt
DeepBSDE.py:326-341), and loss_function (nd_BSPDE_case.py:237-281,
DeepBSDE.py:202-245) calls them inside its time loop.  The native step runs
the coefficients declared by problem_spec() in its kernels; a subclass
without a spec, or whose overridden methods disagree with the spec it
inherits, runs here instead:

  1. X rollout on the device with the subclass's own mu_tf / sigma_tf, the
     reference's expression in its order (valid because mu and sigma do not
     read Y or Z -- checked at construction, `state_independence`), so X does
     not depend on the network;
  2. u and Z = du/dX at all R = M(N+1) rows in ONE native dbsde_net_u (the
     fused HIP forward + input-gradient kernels);
  3. the residual loss from the subclass's phi_tf / g_tf / Dg_tf, step by step
     as the reference writes it (the D == 1 squeeze() broadcast of the
     Y-tilde term included), on detached leaves for u and Z;
  4. torch autograd of that loss gives the cotangents (ubar, zbar) of u and Z
     -- the only way the loss depends on the parameters once X is fixed --
     and ONE native dbsde_net_u_vjp contracts them into d loss / d params.

The network work (steps 2 and 4: forward, input gradient, the double
backward and every weight gradient) is the native HIP path; torch evaluates
the user's coefficient expressions, which are user Python code.  Nothing
here imports the oracle.
"""
from __future__ import annotations

import math

import torch

COEFFICIENTS = ("mu_tf", "sigma_tf", "phi_tf", "g_tf", "Dg_tf")
_PKG = __name__.rsplit(".", 1)[0]


# ---------------------------------------------------------------------- spec formulas
def spec_functions(spec, strike=None):
    """The coefficients a DIAG ProblemSpec declares (include/dbsde.h), as
    torch functions of the reference methods' signatures."""
    K = spec.strike if strike is None else strike

    def cols(X):
        return X[:, :spec.g_cols] if spec.g_cols else X

    def mu(t, X, Y=None, Z=None):
        return spec.mu_a * X

    def sigma(t, X, Y=None):
        return torch.diag_embed(spec.sig_a * X + spec.sig_b)

    def phi(t, X, Y, Z):
        return spec.phi_r * (Y - spec.phi_c * torch.sum(X * Z, dim=1, keepdim=True)) + \
            spec.phi_zz * torch.sum(Z * Z, dim=1, keepdim=True)

    def g(X):
        S = cols(X)
        if spec.g == "sumsq":
            return torch.sum(S ** 2, dim=1, keepdim=True)
        if spec.g == "call_sum":
            return torch.clamp(torch.sum(S, dim=1, keepdim=True) - K, min=0.0)
        if spec.g == "call_mean":
            return torch.clamp(torch.mean(S, dim=1, keepdim=True) - K, min=0.0)
        if spec.g == "log":
            return torch.log(0.5 + 0.5 * torch.sum(S ** 2, dim=1, keepdim=True))
        if spec.g == "smooth_call":
            a = torch.mean(S, dim=1, keepdim=True) - K
            return a / (1 + torch.exp(-spec.g_alpha * a))
        raise ValueError(f"unknown terminal condition {spec.g!r}")

    def dg(X):
        X = X.detach().requires_grad_(True)
        with torch.enable_grad():
            v = g(X)
            return torch.autograd.grad(v, X, torch.ones_like(v))[0]

    return {"mu_tf": mu, "sigma_tf": sigma, "phi_tf": phi, "g_tf": g, "Dg_tf": dg}


def overridden(obj, base, name):
    """The class that defines obj's `name`, if it is not `base`'s."""
    for klass in type(obj).__mro__:
        if name in klass.__dict__:
            return None if klass.__dict__[name] is base.__dict__.get(name) else klass
    return None


def user_defined(klass):
    return klass is not None and not (klass.__module__ or "").startswith(_PKG)


def probe_inputs(D, T, xi, device, P=16, seed=1234):
    """Probe rows (t, X, Y, Z): X positive at scales 1/4..4 of the initial
    state (the region the paths visit), Y and Z standard normal."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    scale = float(torch.as_tensor(xi).detach().abs().max()) if xi is not None else 1.0
    scale = scale if math.isfinite(scale) and scale > 0 else 1.0
    s = scale * torch.logspace(-math.log10(4.0), math.log10(4.0), P).reshape(P, 1)
    X = s * (0.5 + torch.rand(P, D, generator=gen))
    t = T * torch.rand(P, 1, generator=gen)
    Y = torch.randn(P, 1, generator=gen)
    Z = torch.randn(P, D, generator=gen)
    return [v.to(device=device, dtype=torch.float32) for v in (t, X, Y, Z)]


def _close(a, b):
    a, b = torch.as_tensor(a).float(), torch.as_tensor(b).float()
    if a.shape != b.shape:
        try:
            a, b = torch.broadcast_tensors(a, b)
        except RuntimeError:
            return False
    scale = max(1.0, float(b.abs().max())) if b.numel() else 1.0
    return bool(torch.allclose(a, b, rtol=1e-5, atol=1e-6 * scale, equal_nan=True))


def coefficient_mismatches(obj, base, spec, D, T, xi, device):
    """Names of the coefficient methods `obj` overrides (relative to `base`)
    whose values on probe inputs differ from what `spec` declares.  Only DIAG
    specs can be compared; for other kinds a method a user class overrides is
    reported as a mismatch."""
    names = [n for n in COEFFICIENTS if overridden(obj, base, n) is not None]
    if not names:
        return []
    if spec.kind != "diag":
        return [n for n in names if user_defined(overridden(obj, base, n))]
    ref = spec_functions(spec)
    t, X, Y, Z = probe_inputs(D, T, xi, device)
    bad = []
    with torch.no_grad():
        for n in names:
            fn = getattr(obj, n)
            try:
                if n in ("mu_tf", "phi_tf"):
                    got, want = fn(t, X, Y, Z), ref[n](t, X, Y, Z)
                elif n == "sigma_tf":
                    got, want = fn(t, X, Y), ref[n](t, X, Y)
                elif n == "g_tf":
                    got, want = fn(X), ref[n](X)
                else:
                    with torch.enable_grad():
                        got = fn(X.clone())
                    want = ref[n](X)
            except NotImplementedError:
                continue                       # an abstract stub: the spec is the definition
            except Exception:                  # noqa: BLE001 -- cannot be compared: run the method itself
                bad.append(n)
                continue
            if not _close(got, want):
                bad.append(n)
    return bad


def state_independence(obj, D, T, xi, device):
    """Raise ValueError when mu_tf or sigma_tf reads Y or Z.  The
    time-parallel restatement (rollout first, then one batch of network rows)
    needs X independent of the network; the reference's abstract
    mu_tf(t, X, Y, Z) allows a dependence no shipped problem has."""
    t, X, Y, Z = probe_inputs(D, T, xi, device, P=8, seed=99)
    Y = Y.clone().requires_grad_(True)
    Z = Z.clone().requires_grad_(True)
    with torch.enable_grad():
        for name, out in (("mu_tf", obj.mu_tf(t, X, Y, Z)), ("sigma_tf", obj.sigma_tf(t, X, Y))):
            out = torch.as_tensor(out)
            if not out.requires_grad:
                continue
            gs = torch.autograd.grad(out.sum(), (Y, Z), allow_unused=True)
            if any(g is not None and bool((g != 0).any()) for g in gs):
                raise ValueError(
                    f"{type(obj).__name__}.{name} depends on Y or Z: the native solver rolls the paths out "
                    "before evaluating the network (X must not depend on the network parameters)")


# ---------------------------------------------------------------------- the loss
def rollout(fb, t, W, X0):
    """X [M, N+1, D] and sigma(t_n, X_n) dW_n [M, N, D] with the subclass's
    coefficients, nd_BSPDE_case.py:255-258 op for op (mu, sigma never read Y
    or Z here: zeros stand in for them)."""
    M, N1 = t.shape[0], t.shape[1]
    D = X0.shape[1]
    Y0 = torch.zeros((M, 1), device=X0.device)
    Z0 = torch.zeros((M, D), device=X0.device)
    Xs, sdw = [X0], []
    # the increments and time steps of every step at once: the same
    # element-wise fp32 differences the per-step W1 - W0 / t1 - t0 take
    dW = (W[:, 1:, :] - W[:, :-1, :]).unsqueeze(-1)
    dt = t[:, 1:, :] - t[:, :-1, :]
    for n in range(N1 - 1):
        t0 = t[:, n, :]
        s = torch.matmul(fb.sigma_tf(t0, X0, Y0), dW[:, n])
        X1 = X0 + fb.mu_tf(t0, X0, Y0, Z0) * dt[:, n] + torch.squeeze(s, dim=-1)
        sdw.append(s)
        Xs.append(X1)
        X0 = X1
    return torch.stack(Xs, dim=1), sdw


def phi_row_independent(fb, D, device, P=16, seed=4321):
    """True when the subclass's phi_tf treats its rows independently: the
    first P/2 rows of one call over P probe rows equal a call over those rows
    alone.  The reference calls phi_tf once per time step over the M paths;
    a row-wise phi gives the same rows when called once over all M N rows
    (residual_loss's batched form).  A phi that couples rows (a mean over the
    paths, ...) keeps the per-step loop."""
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(P, 1, generator=g)
    X = 0.5 + torch.rand(P, D, generator=g)
    Y = torch.randn(P, 1, generator=g)
    Z = torch.randn(P, D, generator=g)
    t, X, Y, Z = (v.to(device) for v in (t, X, Y, Z))
    h = P // 2
    try:
        with torch.no_grad():
            full = fb.phi_tf(t, X, Y, Z)
            half = fb.phi_tf(t[:h], X[:h], Y[:h], Z[:h])
    except Exception:   # noqa: BLE001 -- anything unusual keeps the reference's loop
        return False
    if not (torch.is_tensor(full) and torch.is_tensor(half) and tuple(full.shape) == (P, 1)
            and tuple(half.shape) == (h, 1)):
        return False
    return bool(torch.allclose(full[:h], half, rtol=1e-5, atol=1e-6))


def residual_loss(fb, t, X, U, DU, sdw, batched=False):
    """nd_BSPDE_case.py:259-275: the residuals of the Euler step of Y and the
    terminal terms, with U [M, N+1, 1] and DU [M, N+1, D] in place of the
    network's outputs (torch.squeeze() of the reference's Y-tilde term kept:
    for D == 1 it broadcasts over the paths).

    batched: phi_tf once over all M N (path, step) rows instead of once per
    step -- the same per-row values for a row-wise phi (phi_row_independent)
    at D > 1, where squeeze() is squeeze(-1); the residual sum then runs in
    one reduction instead of N (a different fp32 summation order).  One
    forward and one backward of a handful of kernels instead of ~N x 40: the
    generic step is bound by those launches."""
    N = t.shape[1] - 1
    M, D = X.shape[0], X.shape[2]
    loss = 0
    if batched and D > 1:
        R = M * N
        S = torch.stack([torch.squeeze(s, dim=-1) for s in sdw], dim=1).reshape(R, D)
        t0, dt = t[:, :N, :].reshape(R, 1), (t[:, 1:, :] - t[:, :N, :]).reshape(R, 1)
        X0, Y0, Z0 = X[:, :N, :].reshape(R, D), U[:, :N, :].reshape(R, 1), DU[:, :N, :].reshape(R, D)
        Y1 = U[:, 1:, :].reshape(R, 1)
        Y1t = Y0 + fb.phi_tf(t0, X0, Y0, Z0) * dt + torch.sum(Z0 * S, dim=1, keepdim=True)
        loss = torch.sum(torch.pow(Y1 - Y1t, 2))
    else:
        for n in range(N):
            t0, t1 = t[:, n, :], t[:, n + 1, :]
            X0, Y0, Z0, Y1 = X[:, n, :], U[:, n, :], DU[:, n, :], U[:, n + 1, :]
            Y1t = Y0 + fb.phi_tf(t0, X0, Y0, Z0) * (t1 - t0) + torch.sum(Z0 * torch.squeeze(sdw[n]), dim=1,
                                                                          keepdim=True)
            loss = loss + torch.sum(torch.pow(Y1 - Y1t, 2))
    XN, YN, ZN = X[:, N, :], U[:, N, :], DU[:, N, :]
    loss = loss + torch.sum(torch.pow(YN - fb.g_tf(XN), 2))
    with torch.enable_grad():
        dg = fb.Dg_tf(XN.detach().requires_grad_(True))
    loss = loss + torch.sum(torch.pow(ZN - dg.detach(), 2))
    return loss


def loss_grad(fb, params, t, W, Xi, grad=None, want=("X", "Y"), loss_out=None):
    """FBSNN.loss_function (+ loss.backward into `grad`) for a subclass
    outside the native coefficient table.  t [M, N+1(, 1)], W [M, N+1, D]
    device fp32; Xi [1 or M, D].  Returns the dict FBSNN._run returns."""
    dev = fb.device
    M, N1 = t.shape[0], t.shape[1]
    D = fb.state_dim
    t = torch.as_tensor(t, dtype=torch.float32).to(dev).reshape(M, N1, 1)
    W = torch.as_tensor(W, dtype=torch.float32).to(dev).reshape(M, N1, -1)
    Xi = torch.as_tensor(Xi, dtype=torch.float32).to(dev).reshape(-1, D)
    X0 = Xi.repeat(M, 1) if Xi.shape[0] == 1 else Xi
    with torch.no_grad():
        X, sdw = rollout(fb, t, W, X0.detach())
    R = M * N1
    trow = t.reshape(R).contiguous()
    xrow = X.reshape(R, D).contiguous()
    u = torch.empty((R, 1), device=dev)
    du = torch.empty((R, D), device=dev)
    fb.solver.net_u(params, trow, xrow, u, du)
    U = u.view(M, N1, 1).detach().requires_grad_(grad is not None)
    DU = du.view(M, N1, D).detach().requires_grad_(grad is not None)
    batched = D > 1 and getattr(fb, "_phi_rowwise", None)
    if D > 1 and batched is None:   # probed once per object
        batched = phi_row_independent(fb, D, dev)
        try:
            fb._phi_rowwise = batched
        except AttributeError:
            pass
    with torch.enable_grad() if grad is not None else torch.no_grad():
        loss = residual_loss(fb, t, X, U, DU, sdw, batched=bool(batched))
        if grad is not None:
            ubar, zbar = torch.autograd.grad(loss, (U, DU), allow_unused=True)
            ubar = torch.zeros_like(U) if ubar is None else ubar
            zbar = torch.zeros_like(DU) if zbar is None else zbar
    if grad is not None:
        fb.solver.net_u_vjp(params, trow, xrow, ubar.reshape(R).contiguous().float(),
                            zbar.reshape(R, D).contiguous().float(), grad)
    out = {"loss": torch.empty(1, device=dev) if loss_out is None else loss_out}
    out["loss"].copy_(loss.detach().reshape(1))
    if "X" in want:
        out["X"] = X
    if "Y" in want:
        out["Y"] = u.view(M, N1, 1)
    if "Z" in want:
        out["Z"] = du.view(M, N1, D)
    return out


__all__ = ["spec_functions", "coefficient_mismatches", "state_independence", "loss_grad", "rollout",
           "residual_loss", "phi_row_independent", "COEFFICIENTS"]
