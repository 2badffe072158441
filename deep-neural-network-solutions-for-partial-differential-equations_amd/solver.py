"""NativeSolver: one C-ABI context (one GPU) driving the HIP deep-BSDE step.

torch is used only as device-memory/stream plumbing: tensors are handed to
the library as raw device pointers (data_ptr) and kernels are enqueued on
torch's current stream.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib


@dataclass(frozen=True)
class ProblemSpec:
    """Coefficients of one reference FBSNN subclass (see include/dbsde.h):
    kind "diag":   mu = mu_a X, sigma = diag(sig_a X + sig_b)
    kind "heston": k-asset Heston (heston_dnnpde.py:587-605) with S-drift mu_a,
                   kappa/theta/sigma/rho, state [S_1..S_k, v_1..v_k]
    phi = phi_r (Y - phi_c X.Z) + phi_zz |Z|^2, g = g_kind(strike, alpha) over
    the first g_cols state columns (0 = all), u_clamp: u = max(net, 0).
    q3: reproduce the D == 1 squeeze broadcast."""

    mu_a: float = 0.0
    sig_a: float = 0.0
    sig_b: float = 0.0
    phi_r: float = 0.0
    phi_c: float = 0.0
    phi_zz: float = 0.0
    g: str = "sumsq"
    strike: float = 0.0
    q3: bool = True
    kind: str = "diag"
    g_cols: int = 0
    g_alpha: float = 0.0
    u_clamp: bool = False
    kappa: float = 0.0
    theta: float = 0.0
    sigma: float = 0.0
    rho: float = 0.0

    def to_c(self):
        if self.g not in _lib.G_KINDS:
            raise ValueError(f"unknown terminal condition {self.g!r}")
        if self.kind not in _lib.PROBLEM_KINDS:
            raise ValueError(f"unknown problem kind {self.kind!r}")
        return _lib.Problem(_lib.PROBLEM_KINDS[self.kind], self.mu_a, self.sig_a, self.sig_b, self.phi_r,
                            self.phi_c, self.phi_zz, _lib.G_KINDS[self.g], self.strike, int(self.q3),
                            int(self.g_cols), self.g_alpha, int(self.u_clamp), self.kappa, self.theta,
                            self.sigma, self.rho)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class NativeSolver:
    """Owns one dbsde_ctx.  All tensors must be float32, contiguous, on `device`."""

    def __init__(self, mode, layers, activation, problem: ProblemSpec, T, device):
        if mode not in _lib.MODES:
            raise ValueError(f"mode {mode!r} is not one of {sorted(_lib.MODES)}")
        if activation not in _lib.ACTIVATIONS:
            raise ValueError(f"activation {activation!r} is not one of {sorted(_lib.ACTIVATIONS)}")
        if len(layers) > 16:
            raise ValueError("at most 16 layer widths are supported")
        self.lib = _lib.load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("the native deep-BSDE path needs a HIP device (torch 'cuda' device)")
        cfg = _lib.Config()
        cfg.mode = _lib.MODES[mode]
        cfg.activation = _lib.ACTIVATIONS[activation]
        cfg.n_layers = len(layers)
        for k, v in enumerate(layers):
            cfg.layers[k] = int(v)
        cfg.problem = problem.to_c()
        cfg.T = float(T)
        cfg.device = self.device.index if self.device.index is not None else torch.cuda.current_device()
        ctx = ctypes.c_void_p()
        _lib.check(self.lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx)))
        self.ctx = ctx
        self.layers = list(layers)
        self.D = layers[0] - 1
        self.nparams = int(self.lib.dbsde_param_count(ctx))
        mask = (ctypes.c_ubyte * self.nparams)()
        _lib.check(self.lib.dbsde_param_used_mask(ctx, mask, self.nparams), ctx)
        self.used_mask = torch.frombuffer(bytearray(mask), dtype=torch.uint8).bool()
        self.nb = int(self.lib.dbsde_brownian_dim(ctx))
        # bit 0: phase kernels, bit 1: weight-gradient kernel in split-bf16 form
        self.matrix_form = int(self.lib.dbsde_matrix_form(ctx))

    def __del__(self):
        ctx = getattr(self, "ctx", None)
        if ctx is not None and ctx.value:
            try:
                self.lib.dbsde_destroy(ctx)
            except Exception:
                pass
            self.ctx = None

    # ------------------------------------------------------------------
    def _check_tensor(self, t, name, numel=None):
        if t is None:
            return
        if not isinstance(t, torch.Tensor) or t.device != self.device or t.dtype != torch.float32:
            raise ValueError(f"{name} must be a float32 tensor on {self.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if numel is not None and t.numel() != numel:
            raise ValueError(f"{name} has {t.numel()} elements, expected {numel}")

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self.lib.dbsde_set_stream(self.ctx, ctypes.c_void_p(s)), self.ctx)

    def _batch_out(self, params, M, N, Xi, t, W, seed, offset, path0, grad, loss, X, Y, Z):
        D = self.D
        self._check_tensor(params, "params", self.nparams)
        self._check_tensor(grad, "grad", self.nparams)
        self._check_tensor(Xi, "Xi")
        if Xi.numel() not in (D, M * D):
            raise ValueError("Xi must hold 1 or M rows of D values")
        self._check_tensor(t, "t", M * (N + 1))
        self._check_tensor(W, "W", M * (N + 1) * self.nb)
        self._check_tensor(loss, "loss", 1)
        self._check_tensor(X, "X", M * (N + 1) * D)
        self._check_tensor(Y, "Y", M * (N + 1))
        self._check_tensor(Z, "Z", M * (N + 1) * D)
        b = _lib.Batch(int(M), int(N), _ptr(t), _ptr(W), int(seed) & (2 ** 64 - 1),
                       int(offset) & (2 ** 64 - 1), int(path0), _ptr(Xi), Xi.numel() // D)
        return b, _lib.Outputs(_ptr(loss), _ptr(X), _ptr(Y), _ptr(Z))

    def loss_grad(self, params, M, N, Xi, t=None, W=None, seed=0, offset=0, path0=0, grad=None, loss=None,
                  X=None, Y=None, Z=None):
        """FBSNN.loss_function (+ loss.backward when grad is given)."""
        b, o = self._batch_out(params, M, N, Xi, t, W, seed, offset, path0, grad, loss, X, Y, Z)
        self._bind_stream()
        _lib.check(self.lib.dbsde_loss_grad(self.ctx, _ptr(params), ctypes.byref(b), _ptr(grad),
                                            ctypes.byref(o)), self.ctx)

    def train_step(self, params, M, N, Xi, grad, m, v, opt, t=None, W=None, seed=0, offset=0, path0=0, loss=None,
                   X=None, Y=None, Z=None):
        """loss_grad + optimizer_step of one process (dbsde_train_step: the
        update is folded into the gradient finalize when it needs no clip, no
        NaN skip and has a device step counter).  opt: the keyword arguments
        of optimizer_step."""
        b, o = self._batch_out(params, M, N, Xi, t, W, seed, offset, path0, grad, loss, X, Y, Z)
        op = self._optim(params, grad, m, v, **opt)
        self._bind_stream()
        _lib.check(self.lib.dbsde_train_step(self.ctx, _ptr(params), ctypes.byref(b), _ptr(grad), _ptr(m), _ptr(v),
                                             ctypes.byref(op), ctypes.byref(o)), self.ctx)

    def prefetch(self, M, N, Xi, seed=0, offset=0, path0=0):
        """Roll out the device-mode batch a later loss_grad(M, N, Xi, seed=...,
        offset=..., path0=...) with the same Xi tensor will consume
        (dbsde_prefetch).  The rollout is held back until the next
        loss_grad / train_step: a step running the two-stream phase pipeline
        issues it on its second stream after its weight-gradient work, any
        other call on an internal stream ordered after the work queued before
        it.  Xi must stay unchanged (and alive) until the batch is consumed
        or prefetch_drop() is called."""
        D = self.D
        self._check_tensor(Xi, "Xi")
        if Xi.numel() not in (D, M * D):
            raise ValueError("Xi must hold 1 or M rows of D values")
        b = _lib.Batch(int(M), int(N), None, None, int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1),
                       int(path0), _ptr(Xi), Xi.numel() // D)
        self._bind_stream()
        _lib.check(self.lib.dbsde_prefetch(self.ctx, ctypes.byref(b)), self.ctx)

    def prefetch_drop(self):
        """Forget pending prefetches (dbsde_prefetch_cancel)."""
        self._bind_stream()
        _lib.check(self.lib.dbsde_prefetch_cancel(self.ctx), self.ctx)

    def net_u(self, params, t, X, u, Du):
        R = X.numel() // self.D
        self._check_tensor(params, "params", self.nparams)
        for name, v, n in (("t", t, R), ("X", X, R * self.D), ("u", u, R), ("Du", Du, R * self.D)):
            self._check_tensor(v, name, n)
        self._bind_stream()
        _lib.check(self.lib.dbsde_net_u(self.ctx, _ptr(params), R, _ptr(t), _ptr(X), _ptr(u), _ptr(Du)),
                   self.ctx)

    def net_u_vjp(self, params, t, X, ubar, zbar, grad):
        """grad <- d/dparams [sum ubar u + sum zbar . Du] at (t, X) (dbsde_net_u_vjp)."""
        R = X.numel() // self.D
        self._check_tensor(params, "params", self.nparams)
        for name, v, n in (("t", t, R), ("X", X, R * self.D), ("ubar", ubar, R), ("zbar", zbar, R * self.D),
                           ("grad", grad, self.nparams)):
            self._check_tensor(v, name, n)
        self._bind_stream()
        _lib.check(self.lib.dbsde_net_u_vjp(self.ctx, _ptr(params), R, _ptr(t), _ptr(X), _ptr(ubar), _ptr(zbar),
                                            _ptr(grad)), self.ctx)

    def optimizer_step(self, params, grad, m, v, **opt):
        """clip_grad_norm_ + optimizer.step() over the flat parameters; m, v are
        the optimizer's state buffers (see include/dbsde.h DBSDE_OPT_*); opt as
        _optim."""
        o = self._optim(params, grad, m, v, **opt)
        self._bind_stream()
        _lib.check(self.lib.dbsde_optimizer_step(self.ctx, _ptr(params), _ptr(grad), _ptr(m), _ptr(v),
                                                 ctypes.byref(o)), self.ctx)

    def _optim(self, params, grad, m, v, kind="Adam", lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
               weight_decay=0.0, max_norm=0.0, step=1, alpha=0.99, rho=0.9, lr_decay=0.0, lambd=1e-4,
               asgd_eta=0.0, asgd_mu=1.0, skip_nonfinite_loss=None, step_state=None, step_parity=0):
        """The dbsde_optim block.  step_state: optional device float64[2] step
        counter (dbsde_optim.step_state): the update number, and from it the
        step-dependent scalars, then come from the device, and a skipped update
        does not advance it."""
        if kind not in _lib.OPTIMIZERS:
            raise ValueError(f"Optimizer type '{kind}' is not recognized.")
        if kind == "ASGD" and step_state is None and not asgd_eta:
            # without the device step counter ASGD's eta / mu come from the
            # caller; eta = 0 would silently leave the parameters unchanged
            raise ValueError("ASGD needs step_state (device step counter) or an explicit asgd_eta > 0")
        for name, v_ in (("params", params), ("grad", grad), ("m", m), ("v", v)):
            self._check_tensor(v_, name, self.nparams)
        self._check_tensor(skip_nonfinite_loss, "loss", 1)
        if step_state is not None and (step_state.device != self.device or step_state.dtype != torch.float64
                                       or step_state.numel() != 2):
            raise ValueError(f"step_state must be a float64 tensor of 2 elements on {self.device}")
        return _lib.Optim(_lib.OPTIMIZERS[kind], lr, betas[0], betas[1], eps, weight_decay,
                          max_norm if max_norm else 0.0, int(step), alpha, rho, lr_decay, lambd, asgd_eta, asgd_mu,
                          _ptr(skip_nonfinite_loss), _ptr(step_state), int(step_parity))

    # ------------------------------------------------------------------ L-BFGS vector primitives
    def vec_reduce(self, op, a, b=None):
        """Fixed-order fp64 sum a.b ("dot"), sum |a| ("asum") or max |a| ("amax")
        of device fp32 vectors, returned as a Python float (syncs)."""
        self._check_tensor(a, "a")
        self._check_tensor(b, "b", a.numel() if b is not None else None)
        out = ctypes.c_double()
        self._bind_stream()
        _lib.check(self.lib.dbsde_vec_reduce(self.ctx, _lib.VEC_OPS[op], _ptr(a), _ptr(b), a.numel(),
                                             ctypes.byref(out)), self.ctx)
        return out.value

    def vec_axpby(self, z, x, alpha, y=None, beta=0.0):
        """z = alpha x + beta y (fp32, on the device)."""
        for name, v in (("z", z), ("x", x), ("y", y)):
            self._check_tensor(v, name, z.numel() if v is not None else None)
        self._bind_stream()
        _lib.check(self.lib.dbsde_vec_axpby(self.ctx, _ptr(z), _ptr(x), _ptr(y), z.numel(), float(alpha),
                                            float(beta)), self.ctx)

    def lbfgs_direction(self, g, S, Y, slots, ro, h_diag, d):
        """torch LBFGS two-loop recursion over history rows `slots` (oldest first)."""
        n = g.numel()
        for name, v in (("g", g), ("d", d)):
            self._check_tensor(v, name, n)
        num = len(slots)
        if num:
            self._check_tensor(S, "S")
            self._check_tensor(Y, "Y", S.numel())
            if S.dim() != 2 or S.shape[1] < n or max(slots) >= S.shape[0]:
                raise ValueError("history matrices must be [slots, >= n] and hold every slot")
        sl = (ctypes.c_int * max(num, 1))(*slots)
        rv = (ctypes.c_float * max(num, 1))(*ro)
        self._bind_stream()
        _lib.check(self.lib.dbsde_lbfgs_direction(self.ctx, _ptr(g), _ptr(S) if num else None,
                                                  _ptr(Y) if num else None, S.shape[1] if num else n, n, sl, rv,
                                                  num, float(h_diag), _ptr(d)), self.ctx)

    # ------------------------------------------------------------------ Brownian increments
    def set_corr(self, L):
        """Cholesky factor for the device mode (None clears), with_corr...py:339-341."""
        if L is None:
            _lib.check(self.lib.dbsde_set_corr(self.ctx, None, 0), self.ctx)
            return
        import numpy as np
        L = np.ascontiguousarray(np.asarray(L, dtype=np.float32))
        if L.shape != (self.nb, self.nb):
            raise ValueError(f"L must be [{self.nb}, {self.nb}]")
        self._bind_stream()
        _lib.check(self.lib.dbsde_set_corr(self.ctx, L.ctypes.data_as(ctypes.c_void_p), self.nb), self.ctx)

    def brownian(self, M, N, seed=0, offset=0, path0=0, increments=False):
        """Device fetch_minibatch: (t [M, N+1], W [M, N+1, nb]) or, with
        increments=True, (t, dW [M, N, nb]) as the device-mode rollout draws them."""
        t = torch.empty((M, N + 1), device=self.device)
        W = torch.empty((M, N if increments else N + 1, self.nb), device=self.device)
        xi = torch.zeros(self.D, device=self.device)
        b = _lib.Batch(int(M), int(N), None, None, int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1),
                       int(path0), _ptr(xi), 1)
        self._bind_stream()
        _lib.check(self.lib.dbsde_brownian(self.ctx, ctypes.byref(b), _ptr(t), _ptr(W), int(increments)), self.ctx)
        return t, W

    # ------------------------------------------------------------------ profiling
    def profile(self, enable=True):
        _lib.check(self.lib.dbsde_profile_enable(self.ctx, int(enable)), self.ctx)

    def profile_reset(self):
        _lib.check(self.lib.dbsde_profile_reset(self.ctx), self.ctx)

    def profile_read(self):
        n = self.lib.dbsde_profile_count(self.ctx)
        if n < 0:
            _lib.check(n, self.ctx)
        out = {}
        name = ctypes.create_string_buffer(128)
        ms, fl, by, nl = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
        for i in range(n):
            _lib.check(self.lib.dbsde_profile_read(self.ctx, i, name, 128, ctypes.byref(ms), ctypes.byref(fl),
                                                   ctypes.byref(by), ctypes.byref(nl)), self.ctx)
            out[name.value.decode()] = dict(ms=ms.value, flops=fl.value, bytes=by.value, launches=nl.value)
        return out


# ---------------------------------------------------------------------- evaluators
def exact(kind, t, X, T, params):
    """Device exact / comparator solutions (include/dbsde.h dbsde_exact):
    kind in {"bsb", "bs_call", "basket_avg", "basket_mean"}; t [R], X [R, D]
    float32 cuda tensors.  Returns (price, delta); delta is None for "bsb"."""
    lib = _lib.load()
    if kind not in _lib.EXACT_KINDS:
        raise ValueError(f"unknown exact solution {kind!r}")
    X = X.reshape(X.shape[0], -1).contiguous().float()
    t = t.reshape(-1).contiguous().float()
    R, D = X.shape
    if t.numel() != R or X.device.type != "cuda" or t.device != X.device:
        raise ValueError("t [R] and X [R, D] must be float32 tensors on the same HIP device")
    ncol = D if kind == "bs_call" else 1
    price = torch.empty((R, ncol), device=X.device)
    delta = None if kind == "bsb" else torch.empty((R, ncol), device=X.device)
    import numpy as np
    p = np.zeros(3, dtype=np.float64)
    p[:len(params)] = params
    s = torch.cuda.current_stream(X.device).cuda_stream
    _lib.check(lib.dbsde_exact(_lib.EXACT_KINDS[kind], _ptr(t), _ptr(X), R, D, float(T),
                               p.ctypes.data_as(ctypes.c_void_p), _ptr(price), _ptr(delta), ctypes.c_void_p(s)))
    return price, delta


def hjb_mc(t, X, T, mc=10 ** 5, seed=0):
    """HJB Monte-Carlo value (hjb_implement.py:1088-1095) at P points."""
    lib = _lib.load()
    X = X.reshape(X.shape[0], -1).contiguous().float()
    t = t.reshape(-1).contiguous().float()
    P, D = X.shape
    if t.numel() != P or X.device.type != "cuda" or t.device != X.device:
        raise ValueError("t [P] and X [P, D] must be float32 tensors on the same HIP device")
    u = torch.empty((P, 1), device=X.device)
    s = torch.cuda.current_stream(X.device).cuda_stream
    _lib.check(lib.dbsde_hjb_mc(_ptr(t), _ptr(X), P, D, float(T), int(mc), int(seed) & (2 ** 64 - 1), _ptr(u),
                                ctypes.c_void_p(s)))
    return u
