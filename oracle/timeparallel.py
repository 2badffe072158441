"""ORACLE -- test infrastructure only, never the product path.

NumPy (float64 by default) statement of the *time-parallel* form of the
deep-BSDE loss and its parameter gradient -- the algorithm the HIP kernels
implement -- derived by hand from the reference graph:

  * X does not depend on the network (mu, sigma never read Y or Z in any
    reference problem: DeepBSDE.py:337-341, nd_BSPDE_case.py:524-539,
    hjb_implement.py:600-604, with_corr...:581-596), so the Euler-Maruyama
    rollout (DeepBSDE.py:218-222) is computed first and all M*(N+1) network
    evaluations become one batch of rows.
  * Z = du/dx is the input-gradient pass (DeepBSDE.py:189-194).
  * The loss (DeepBSDE.py:223-240) is a sum of squared residuals whose
    cotangents (ubar for Y, zbar for Z) are closed form.
  * d/dtheta [ubar*u + zbar.grad_x u] = reverse mode over (primal forward +
    forward tangent along zbar) -- SURVEY 3.3.

Checked against the reference's golden vectors in tests/test_oracle_golden.py
(and thereby against fbsnn_ref's autograd double backward).

Unified network ("blocks"): every supported mode is
    h_1 = act(x W_in^T + b_in)
    a_k = h_k B_k^T + [x V_k^T] + beta_k,   h_{k+1} = act(a_k) + rho*h_k,   k=1..K
    u   = h_{K+1} . w_out + b_out
  NAIS-Net / Naisnet: B_k = -A_k (A_k = proj(W_k), Q4), V_k present, rho=1
  Resnet:             B_k = W_k, no V_k, rho=1
  FC:                 B_k = W_k, no V_k, rho=0
"""
from __future__ import annotations

import numpy as np

# --------------------------------------------------------------------------
# parameter layout (state_dict order of the reference modules)
# --------------------------------------------------------------------------


def param_layout(mode, layers):
    """[(name, shape)] in reference state_dict order (SURVEY 8(b) layout row)."""
    L = list(layers)
    out = []
    if mode == "FC":
        for i in range(len(L) - 1):
            out += [(f"{2 * i}.weight", (L[i + 1], L[i])), (f"{2 * i}.bias", (L[i + 1],))]
    elif mode in ("NAIS-Net", "Resnet"):
        out += [("input_layer.weight", (L[1], L[0])), ("input_layer.bias", (L[1],))]
        for i in range(1, len(L) - 2):
            out += [(f"hidden_layers.{i - 1}.weight", (L[i + 1], L[i])),
                    (f"hidden_layers.{i - 1}.bias", (L[i + 1],))]
        out += [("output_layer.weight", (L[-1], L[-2])), ("output_layer.bias", (L[-1],))]
        if mode == "NAIS-Net":
            for i in range(1, len(L) - 1):
                out += [(f"input_layers.{i - 1}.weight", (L[i], L[0])),
                        (f"input_layers.{i - 1}.bias", (L[i],))]
    elif mode == "Naisnet":
        n = len(L)
        out += [("layer1.weight", (L[1], L[0])), ("layer1.bias", (L[1],)),
                ("layer2.weight", (L[2], L[1])), ("layer2.bias", (L[2],)),
                ("layer2_input.weight", (L[2], L[0])), ("layer2_input.bias", (L[2],)),
                ("layer3.weight", (L[3], L[2])), ("layer3.bias", (L[3],))]
        if n >= 5:
            out += [("layer3_input.weight", (L[3], L[0])), ("layer3_input.bias", (L[3],)),
                    ("layer4.weight", (L[4], L[3])), ("layer4.bias", (L[4],))]
        if n == 6:
            out += [("layer4_input.weight", (L[4], L[0])), ("layer4_input.bias", (L[4],)),
                    ("layer5.weight", (L[5], L[4])), ("layer5.bias", (L[5],))]
    else:
        raise ValueError(mode)
    return out


def unpack(flat, mode, layers):
    d, off = {}, 0
    for name, shp in param_layout(mode, layers):
        n = int(np.prod(shp))
        d[name] = np.asarray(flat[off:off + n]).reshape(shp)
        off += n
    assert off == len(flat)
    return d


def _names(mode, layers):
    """Map the unified blocks onto parameter names.
    Returns dict(in_w, in_b, blocks=[(B_w, B_b, V_w|None, V_b|None)], out_w, out_b, rho, proj)."""
    K = len(layers) - 3
    if mode == "FC":
        blocks = [(f"{2 * k}.weight", f"{2 * k}.bias", None, None) for k in range(1, K + 1)]
        return dict(in_w="0.weight", in_b="0.bias", blocks=blocks,
                    out_w=f"{2 * (K + 1)}.weight", out_b=f"{2 * (K + 1)}.bias", rho=0.0, proj=False)
    if mode in ("NAIS-Net", "Resnet"):
        st = mode == "NAIS-Net"
        blocks = [(f"hidden_layers.{k}.weight", f"hidden_layers.{k}.bias",
                   f"input_layers.{k}.weight" if st else None,
                   f"input_layers.{k}.bias" if st else None) for k in range(K)]
        return dict(in_w="input_layer.weight", in_b="input_layer.bias", blocks=blocks,
                    out_w="output_layer.weight", out_b="output_layer.bias", rho=1.0, proj=st)
    if mode == "Naisnet":
        blocks = [(f"layer{k + 2}.weight", f"layer{k + 2}.bias",
                   f"layer{k + 2}_input.weight", f"layer{k + 2}_input.bias") for k in range(K)]
        return dict(in_w="layer1.weight", in_b="layer1.bias", blocks=blocks,
                    out_w=f"layer{K + 2}.weight", out_b=f"layer{K + 2}.bias", rho=1.0, proj=True)
    raise ValueError(mode)


# --------------------------------------------------------------------------
# activations
# --------------------------------------------------------------------------


def act_fns(name):
    if name == "Sine":
        return np.sin, np.cos, lambda a: -np.sin(a)
    if name == "Tanh":
        def d1(a):
            return 1.0 - np.tanh(a) ** 2

        def d2(a):
            th = np.tanh(a)
            return -2.0 * th * (1.0 - th * th)
        return np.tanh, d1, d2
    if name == "ReLU":
        return (lambda a: np.maximum(a, 0.0), lambda a: (a > 0).astype(a.dtype),
                lambda a: np.zeros_like(a))
    raise ValueError(name)


# --------------------------------------------------------------------------
# NAIS projection and its adjoint (Q4)
# --------------------------------------------------------------------------


def project(Wk, eps=0.01):
    delta = 1 - 2 * eps
    R = Wk.T @ Wk
    n = np.sqrt(np.sum(R * R))
    s = np.sqrt(delta) / np.sqrt(n) if n > delta else 1.0
    return s * R + eps * np.eye(R.shape[0]), (R, n, s, n > delta)


def project_vjp(Wk, Abar, aux, eps=0.01):
    """Given Abar = dL/dA, return dL/dW for A = proj(W)."""
    R, n, s, taken = aux
    if taken:
        delta = 1 - 2 * eps
        Rbar = np.sqrt(delta) * n ** -0.5 * (Abar - 0.5 * np.sum(Abar * R) * R / (n * n))
    else:
        Rbar = Abar
    return Wk @ (Rbar + Rbar.T)


# --------------------------------------------------------------------------
# problem coefficients in parametric form (one row = one (path, time) pair)
# --------------------------------------------------------------------------

PROBLEMS = {
    #            mu_a  sig_a sig_b        phi_r phi_c phi_zz  g
    "bsb":        (0.0, 0.4, 0.0,          0.05, 1.0, 0.0, "sumsq"),
    "bspde_test": (0.05, 0.2, 0.0,         0.05, 1.0, 0.0, "sumsq"),
    "call":       (0.05, 0.2, 0.0,         0.05, 1.0, 0.0, "call_sum"),
    "call1d":     (0.01, 0.25, 0.0,        0.01, 0.0, 0.0, "call_sum"),
    "basket":     (0.05, 0.2, 0.0,         0.05, 0.0, 0.0, "call_mean"),
    "hjb":        (0.0, 0.0, np.sqrt(2.0), 0.0, 0.0, 1.0, "log"),
}


HESTON_DEFAULTS = dict(kappa=2.0, theta=0.2, sigma=0.3, rho=0.8, v0=0.2, payoff="discontinuous")


def g_and_grad(kind, X, strike):
    if kind == "sumsq":
        return np.sum(X * X, 1), 2.0 * X
    if kind == "call_sum":
        s = np.sum(X, 1) - strike
        return np.maximum(s, 0.0), np.repeat((s > 0).astype(X.dtype)[:, None], X.shape[1], 1)
    if kind == "call_mean":
        s = np.mean(X, 1) - strike
        return np.maximum(s, 0.0), np.repeat((s > 0).astype(X.dtype)[:, None], X.shape[1], 1) / X.shape[1]
    if kind == "log":
        q = 0.5 + 0.5 * np.sum(X * X, 1)
        return np.log(q), X / q[:, None]
    if kind == "smooth_call":       # heston_dnnpde.py:551-556: a / (1 + e^{-10 a}), a = mean X - K
        a = np.mean(X, 1) - strike
        e = np.exp(-10.0 * a)
        d = (1.0 / (1.0 + e) + a * 10.0 * e / (1.0 + e) ** 2) / X.shape[1]
        return a / (1.0 + e), np.repeat(d[:, None], X.shape[1], 1)
    raise ValueError(kind)


def heston_rollout(t, W, Xi, kappa, theta, sigma, rho, **_):
    """heston_dnnpde.py:629-642 (fp64): state [S_1..S_k, v_1..v_k], W [M, N+1, k];
    sdw is the vector the Y-tilde term contracts with Z."""
    M, N1, k = W.shape
    X = np.zeros((M, N1, 2 * k))
    X[:, 0] = Xi if Xi.shape[0] == M else np.repeat(Xi.reshape(1, 2 * k), M, 0)
    sdw = np.zeros((M, N1 - 1, 2 * k))
    c = lambda a: np.clip(a, -100.0, 100.0)
    for n in range(N1 - 1):
        S, v = X[:, n, :k], X[:, n, k:]
        dt = (t[:, n + 1] - t[:, n])[:, None]
        w = W[:, n + 1] - W[:, n]
        sv = np.sqrt(np.maximum(v, 1e-8))
        d00, d11, d01, d10 = c(sv * S), c(sigma * sv), c(rho * sigma * sv), c(rho * sv * S)
        sdw[:, n, :k] = (d00 + d01) * w
        sdw[:, n, k:] = (d10 + d11) * w
        X[:, n + 1, :k] = S + c(0.05 * S) * dt + sdw[:, n, :k]
        X[:, n + 1, k:] = v + c(kappa * (theta - v)) * dt + sdw[:, n, k:]
    return X, sdw


def rollout(problem, t, W, Xi):
    """Euler-Maruyama X path (DeepBSDE.py:218-222) and sigma*dW per step."""
    mu_a, sig_a, sig_b = PROBLEMS[problem][:3]
    M, N1, D = W.shape
    X = np.zeros((M, N1, D), dtype=W.dtype)
    X[:, 0] = Xi if Xi.shape[0] == M else np.repeat(Xi.reshape(1, D), M, 0)
    sdw = np.zeros((M, N1 - 1, D), dtype=W.dtype)
    for n in range(N1 - 1):
        x0 = X[:, n]
        dt = t[:, n + 1] - t[:, n]
        s = (sig_a * x0 + sig_b) * (W[:, n + 1] - W[:, n])
        X[:, n + 1] = x0 + mu_a * x0 * dt + s
        sdw[:, n] = s
    return X, sdw


# --------------------------------------------------------------------------
# the time-parallel loss / gradient
# --------------------------------------------------------------------------


def loss_grad(flat, mode, layers, activation, problem, t, W, Xi, strike=None, q3=True, heston=None):
    """Returns dict(loss, X, Y, Z, grad) with grad in state_dict order (unused
    Q6 parameters get 0).  problem == "heston": the k-asset Heston problem
    (heston_dnnpde.py:519-659) with parameters `heston` (HESTON_DEFAULTS), Xi
    the full initial state [S, v], W [M, N+1, k]."""
    P = unpack(flat, mode, layers)
    nm = _names(mode, layers)
    sig, d1, d2 = act_fns(activation)
    D = layers[0] - 1
    t = np.asarray(t)
    if t.ndim == 3:
        t = t[:, :, 0]
    M, N1, _ = W.shape
    N = N1 - 1
    clamp = problem == "heston"
    if clamp:
        hp = dict(HESTON_DEFAULTS, **(heston or {}))
        mu_a, sig_a, sig_b, phi_r, phi_c, phi_zz = 0.05, 0.0, 0.0, 0.05, 0.0, 0.0
        gk = "call_mean" if hp["payoff"] == "discontinuous" else "smooth_call"
        G = D // 2
        strike = 1.0 if strike is None else strike
        X, sdw = heston_rollout(t, W, Xi, **hp)
        q3 = False
    else:
        mu_a, sig_a, sig_b, phi_r, phi_c, phi_zz, gk = PROBLEMS[problem]
        G = D
        if strike is None:
            strike = {"call": 1.0 * D, "call1d": 1.0 * D, "basket": 1.0}.get(problem, 0.0)
        X, sdw = rollout(problem, t[:, :, None], W, Xi)
    R = M * N1
    x = np.concatenate([t.reshape(R, 1), X.reshape(R, D)], 1)          # [R, D+1]

    Win, bin_ = P[nm["in_w"]], P[nm["in_b"]]
    Bs, betas, Vs, As_aux = [], [], [], []
    for (bw, bb, vw, vb) in nm["blocks"]:
        Wk = P[bw]
        if nm["proj"]:
            A, aux = project(Wk)
            Bs.append(-A)
            As_aux.append(aux)
        else:
            Bs.append(Wk)
            As_aux.append(None)
        beta = P[bb] + (P[vb] if vb is not None else 0.0)
        betas.append(beta)
        Vs.append(P[vw] if vw is not None else None)
    wout, bout = P[nm["out_w"]][0], P[nm["out_b"]][0]
    rho = nm["rho"]
    K = len(Bs)

    # ---- primal forward
    a = [x @ Win.T + bin_]
    h = [None, sig(a[0])]                      # h[1]
    for k in range(K):
        ak = h[k + 1] @ Bs[k].T + betas[k]
        if Vs[k] is not None:
            ak = ak + x @ Vs[k].T
        a.append(ak)
        h.append(sig(ak) + rho * h[k + 1])     # h[k+2] = h_{k+2}
    u = h[K + 1] @ wout + bout
    umask = np.ones_like(u)
    if clamp:                                   # heston_dnnpde.py:568, clamp passes the gradient at 0
        umask = (u >= 0).astype(u.dtype)
        u = u * umask

    # ---- input gradient (delta[k] pairs with a[k])
    g = [None] * (K + 2)
    delta = [None] * (K + 1)
    g[K + 1] = np.broadcast_to(wout, (R, wout.shape[0]))
    for k in range(K, 0, -1):
        delta[k] = g[k + 1] * d1(a[k])
        g[k] = rho * g[k + 1] + delta[k] @ Bs[k - 1]
    delta[0] = g[1] * d1(a[0])
    zfull = delta[0] @ Win
    for k in range(1, K + 1):
        if Vs[k - 1] is not None:
            zfull = zfull + delta[k] @ Vs[k - 1]
    Z = zfull[:, 1:] * umask[:, None]

    # ---- residuals and cotangents
    Y = u.reshape(M, N1)
    Zr = Z.reshape(M, N1, D)
    dt = t[:, 1:] - t[:, :-1]
    s_xz = np.sum(X[:, :-1] * Zr[:, :-1], 2)
    s_zz = np.sum(Zr[:, :-1] ** 2, 2)
    if D == 1 and q3:
        s_zs = Zr[:, :-1, 0] * np.sum(sdw[:, :, 0], 0)[None, :]
    else:
        s_zs = np.sum(Zr[:, :-1] * sdw, 2)
    phi = phi_r * (Y[:, :-1] - phi_c * s_xz) + phi_zz * s_zz
    ytil = Y[:, :-1] + phi * dt + s_zs
    r = Y[:, 1:] - ytil                                             # [M, N]
    gT, dgT = g_and_grad(gk, X[:, -1, :G], strike)
    rT = Y[:, -1] - gT
    zT = Zr[:, -1, :G] - dgT
    loss = np.sum(r * r) + np.sum(rT * rT) + np.sum(zT * zT)

    ubar = np.zeros((M, N1))
    ubar[:, 1:] += 2 * r
    ubar[:, :-1] += -2 * r * (1 + phi_r * dt)
    ubar[:, -1] += 2 * rT
    zb = np.zeros((M, N1, D))
    dphidz = -phi_r * phi_c * X[:, :-1] + 2 * phi_zz * Zr[:, :-1]
    if D == 1 and q3:
        dsz = np.broadcast_to(np.sum(sdw[:, :, 0], 0)[None, :, None], sdw.shape)
    else:
        dsz = sdw
    zb[:, :-1] = -2 * r[:, :, None] * (dphidz * dt[:, :, None] + dsz)
    zb[:, -1, :G] = 2 * zT
    ub = ubar.reshape(R) * umask
    zb = zb * umask.reshape(M, N1, 1)
    zbar = np.concatenate([np.zeros((R, 1)), zb.reshape(R, D)], 1)   # t-component 0

    # ---- forward tangent along zbar
    adot = [zbar @ Win.T]
    hdot = [None, d1(a[0]) * adot[0]]
    for k in range(K):
        ad = hdot[k + 1] @ Bs[k].T
        if Vs[k] is not None:
            ad = ad + zbar @ Vs[k].T
        adot.append(ad)
        hdot.append(d1(a[k + 1]) * ad + rho * hdot[k + 1])

    # ---- reverse over (primal, tangent)
    grads = {n: np.zeros(s) for n, s in param_layout(mode, layers)}
    grads[nm["out_w"]][0] = ub @ h[K + 1] + np.sum(hdot[K + 1], 0)
    grads[nm["out_b"]][0] = np.sum(ub)
    p = ub[:, None] * wout[None, :]                                  # p_{K+1}
    for k in range(K, 0, -1):
        alpha = p * d1(a[k]) + g[k + 1] * adot[k] * d2(a[k])
        bw, bb, vw, vb = nm["blocks"][k - 1]
        Bbar = alpha.T @ h[k] + delta[k].T @ hdot[k]
        if nm["proj"]:
            grads[bw] += project_vjp(P[bw], -Bbar, As_aux[k - 1])
        else:
            grads[bw] += Bbar
        grads[bb] += np.sum(alpha, 0)
        if vw is not None:
            grads[vw] += alpha.T @ x + delta[k].T @ zbar
            grads[vb] += np.sum(alpha, 0)
        p = rho * p + alpha @ Bs[k - 1]
    alpha0 = p * d1(a[0]) + g[1] * adot[0] * d2(a[0])
    grads[nm["in_w"]] += alpha0.T @ x + delta[0].T @ zbar
    grads[nm["in_b"]] += np.sum(alpha0, 0)

    flatg = np.concatenate([grads[n].reshape(-1) for n, _ in param_layout(mode, layers)])
    return dict(loss=loss, X=X, Y=Y[:, :, None], Z=Zr, grad=flatg, ubar=ub, zbar=zbar, r=r)


__all__ = ["param_layout", "unpack", "act_fns", "project", "project_vjp", "PROBLEMS", "HESTON_DEFAULTS",
           "g_and_grad", "rollout", "heston_rollout", "loss_grad"]
