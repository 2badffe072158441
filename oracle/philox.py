"""ORACLE -- test infrastructure only, never the product path.

NumPy restatement of the device-mode Brownian increments and path step of the
HIP library (throughput mode, dbsde_batch.W == NULL; csrc/philox.hpp,
csrc/paths.hpp rollout_kernel / rollout_corr_kernel / rollout_heston_kernel,
dbsde_brownian):

  * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as
    easy as 1, 2, 3", SC'11; the Random123 round constants), counter
    (d, n/4, global path, offset), key (seed ^ offset_hi, seed_hi), pinned by
    the Random123 known-answer vectors (tests/test_oracle_philox.py);
  * Box-Muller on the two uniform pairs of one block: four N(0, 1) draws,
    the increments of steps n..n+3 of coordinate d;
  * dW = sqrt(dt) z, or the Cholesky-correlated dW = L (sqrt(dt) z) of
    with_corr_high_dimension_pde.py:334-341;
  * the time grid of the reference's fetch_minibatch: t_n = fp32(fp64 cumsum
    of T/N) (DeepBSDE.py:250-258);
  * the Euler-Maruyama rollout in the reference's operation order
    (DeepBSDE.py:218-222 with sigma = diag(sig_a X + sig_b), mu = mu_a X;
    heston_dnnpde.py:629-642 for the k-asset Heston state), in float32 like
    the kernel.

The reference draws its increments from numpy's legacy normal stream
(DeepBSDE.py:255); no device generator reproduces that stream, so the device
mode is pinned here instead (tests/test_gpu_device_rng.py).  Also the HJB
Monte-Carlo value (hjb_implement.py:1088-1095) on the same draws as the
device comparator (csrc/evals.hip hjb_mc_kernel).
"""
from __future__ import annotations

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_LO = np.uint64(0xFFFFFFFF)
HJB_TAG = 0x484A42          # csrc/evals.hip hjb_mc_kernel counter word


def philox4x32_10(ctr, key):
    """ctr: four uint32 arrays (broadcastable), key: two -> four uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32) for c in ctr)
    k0, k1 = (np.asarray(k, dtype=np.uint32) for k in key)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _LO).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _LO).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + _W0).astype(np.uint32)
            k1 = (k1 + _W1).astype(np.uint32)
    return c0, c1, c2, c3


def normal4(seed, offset, m, nq, d):
    """The four normals of counter (d, nq, m, offset): array [..., 4]."""
    seed, offset = int(seed), int(offset)
    m, nq, d = np.broadcast_arrays(np.asarray(m, np.uint32), np.asarray(nq, np.uint32), np.asarray(d, np.uint32))
    key = (np.uint32((seed ^ (offset >> 32)) & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF))
    c = philox4x32_10((d, nq, m, np.full(d.shape, offset & 0xFFFFFFFF, np.uint32)), key)
    f = 1.0 / 16777216.0
    u1 = ((c[0] >> 8).astype(np.float64) + 1.0) * f
    u2 = (c[1] >> 8).astype(np.float64) * f
    u3 = ((c[2] >> 8).astype(np.float64) + 1.0) * f
    u4 = (c[3] >> 8).astype(np.float64) * f
    r1, r2 = np.sqrt(-2.0 * np.log(u1)), np.sqrt(-2.0 * np.log(u3))
    return np.stack([r1 * np.cos(2 * np.pi * u2), r1 * np.sin(2 * np.pi * u2),
                     r2 * np.cos(2 * np.pi * u4), r2 * np.sin(2 * np.pi * u4)], -1)


def increments(seed, offset, path0, M, N, D, T, L=None):
    """dW [M, N, D] float32 of the device mode for paths path0 .. path0+M-1."""
    m = path0 + np.arange(M)
    nb = (N + 3) // 4
    z = normal4(seed, offset, m[:, None, None], np.arange(nb)[None, :, None], np.arange(D)[None, None, :])
    z = z.transpose(0, 1, 3, 2).reshape(M, 4 * nb, D)[:, :N].astype(np.float32)   # step 4q+k <- z[..., k]
    sq = np.sqrt(np.float32(T) / np.float32(N))
    dw = (sq * z).astype(np.float32)
    if L is not None:
        dw = np.einsum("ij,mnj->mni", np.asarray(L, np.float64), dw.astype(np.float64)).astype(np.float32)
    return dw


def time_grid(N, T):
    """t_n = fp32(fp64 cumsum of T/N), the reference's fetch_minibatch grid."""
    return np.concatenate([[0.0], np.cumsum(np.full(N, T / N))]).astype(np.float32)


def brownian_W(dw):
    """W [M, N+1, nb] = fp32(fp64 cumsum of dW) with W_0 = 0 (dbsde_brownian)."""
    M, N, nb = dw.shape
    W = np.zeros((M, N + 1, nb))
    W[:, 1:] = np.cumsum(dw.astype(np.float64), axis=1)
    return W.astype(np.float32)


def rollout(Xi, dw, T, mu_a=0.0, sig_a=0.0, sig_b=0.0):
    """X [M, N+1, D] float32: x1 = (x + (mu_a x) dt) + (sig_a x + sig_b) dw on the
    reference grid."""
    M, N, D = dw.shape
    f32 = np.float32
    x = np.broadcast_to(np.asarray(Xi, f32).reshape(-1, D), (M, D)).astype(f32)
    X = np.empty((M, N + 1, D), f32)
    tg = time_grid(N, T)
    for n in range(N):
        X[:, n] = x
        dt = f32(tg[n + 1] - tg[n])
        s = (f32(sig_a) * x + f32(sig_b)) * dw[:, n]
        x = (x + (f32(mu_a) * x) * dt) + s
    X[:, N] = x
    return X


def heston_rollout(Xi, dw, T, mu_a=0.05, kappa=2.0, theta=0.2, sigma=0.3, rho=0.8):
    """k-asset Heston state [S_1..S_k, v_1..v_k] (heston_dnnpde.py:587-605,
    629-642): mu and the diffusion blocks clamped to [-100, 100], one dW per
    asset; the X update uses (Sig_i0 + Sig_i1) dW (torch.einsum sums the
    broadcast dimension first).  Returns X [M, N+1, 2k] and the Y-tilde vector
    sdw [M, N, 2k] = (Sig_i0 dW + Sig_i1 dW)."""
    M, N, k = dw.shape
    f32 = np.float32
    x = np.broadcast_to(np.asarray(Xi, f32).reshape(-1, 2 * k), (M, 2 * k)).astype(f32)
    S, v = x[:, :k].copy(), x[:, k:].copy()
    X = np.empty((M, N + 1, 2 * k), f32)
    sdw = np.empty((M, N, 2 * k), f32)
    tg = time_grid(N, T)
    c = lambda a: np.clip(a, f32(-100), f32(100))
    for n in range(N):
        X[:, n, :k], X[:, n, k:] = S, v
        dt = f32(tg[n + 1] - tg[n])
        muS, muV = c(f32(mu_a) * S), c(f32(kappa) * (f32(theta) - v))
        sv = np.sqrt(np.maximum(v, f32(1e-8)))
        sS, sV = sv * S, f32(sigma) * sv
        d00, d11, d01, d10 = c(sS), c(sV), c(f32(rho) * sV), c(f32(rho) * sS)
        w = dw[:, n]
        sdw[:, n, :k] = d00 * w + d01 * w
        sdw[:, n, k:] = d10 * w + d11 * w
        S = (S + muS * dt) + (d00 + d01) * w
        v = (v + muV * dt) + (d10 + d11) * w
    X[:, N, :k], X[:, N, k:] = S, v
    return X, sdw


def hjb_value(t, X, T, mc, seed):
    """hjb_implement.py:1088-1095 on the device comparator's draws:
    -log mean_k 2 / (1 + |X_p + sqrt(2 |T - t_p|) W_k|^2)."""
    t = np.asarray(t, np.float64).reshape(-1)
    X = np.asarray(X, np.float64).reshape(t.size, -1)
    D = X.shape[1]
    nq = (D + 3) // 4
    out = np.empty(t.size)
    for p in range(t.size):
        k = np.arange(mc)
        z = normal4(seed, p, k[:, None], HJB_TAG, np.arange(nq)[None, :]).reshape(mc, 4 * nq)[:, :D]
        s = np.sqrt(2.0 * abs(T - t[p]))
        y = X[p][None, :] + s * z
        out[p] = -np.log(np.mean(2.0 / (1.0 + np.sum(y * y, 1))))
    return out[:, None]


__all__ = ["philox4x32_10", "normal4", "increments", "time_grid", "brownian_W", "rollout", "heston_rollout",
           "hjb_value", "HJB_TAG"]
