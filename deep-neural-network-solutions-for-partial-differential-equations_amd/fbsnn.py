"""FBSNN: the reference solver class surface, driven by the HIP library.

Drop-in for the FBSNN classes of nd_BSPDE_case.py:126-500 (v2: Mm schedule,
optimizer menu, grad clipping, min-loss tracking, save/load),
with_corr_high_dimension_pde.py:132-540 (v3: correlated increments) and,
via deepbsde.FBSNN, DeepBSDE.py:140-323.  Same constructor arguments, method
names, return types and attribute names; the work runs in the C ABI of
include/dbsde.h (one context per GPU).  Subclasses declare their problem
coefficients with `problem_spec()` (see problems.py) and then run them in
the kernels; a subclass that only overrides phi_tf/g_tf/mu_tf/sigma_tf (the
reference's plugin API, nd_BSPDE_case.py:458-500), or overrides one that its
inherited spec does not describe, runs its own methods through generic.py
(its coefficients in torch, the network and the whole backward natively).

Multi-GPU: when torch.distributed is initialised (one process per GPU), the
M paths of every minibatch are split into contiguous blocks of M/world per
rank; gradients and loss are summed with one all-reduce per step and the
optimizer runs replicated.  In parity mode every rank draws the
same global numpy batch (the reference's stream) and uploads only its slice;
in device mode the Philox stream is keyed by the global path index.
"""
from __future__ import annotations

import os
import time
import warnings
from abc import ABC

import numpy as np
import torch
import torch.distributed as dist

from . import generic, networks
from .solver import NativeSolver, ProblemSpec

OPTIMIZER_NAMES = ("Adam", "SGD", "RMSprop", "AdamW", "Adadelta", "Adagrad", "Adamax", "ASGD", "LBFGS")
NATIVE_OPTIMIZERS = OPTIMIZER_NAMES
# torch.optim defaults of each optimizer as the reference builds it, optim.X(params, lr=lr)
# (nd_BSPDE_case.py:331-350; torch 2.10 signatures)
OPT_DEFAULTS = {
    "Adam": dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0),
    "AdamW": dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2),
    "SGD": dict(weight_decay=0.0),
    "RMSprop": dict(alpha=0.99, eps=1e-8, weight_decay=0.0),
    "Adagrad": dict(eps=1e-10, lr_decay=0.0, weight_decay=0.0),
    "Adamax": dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0),
    "Adadelta": dict(rho=0.9, eps=1e-6, weight_decay=0.0),
    "ASGD": dict(lambd=1e-4, alpha=0.75, t0=1e6, weight_decay=0.0),
}


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("the native deep-BSDE path needs a HIP device; none is visible")
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", torch.cuda.current_device())))


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class _NetU(torch.autograd.Function):
    """FBSNN.net_u as a differentiable op: forward dbsde_net_u, backward the
    native VJP dbsde_net_u_vjp (parameter gradients of sum ubar u + zbar . Du),
    split into the model parameters."""

    @staticmethod
    def forward(ctx, fb, t, X, *params):
        u = torch.empty((X.shape[0], 1), device=X.device)
        du = torch.empty_like(X)
        fb.solver.net_u(fb.params, t, X, u, du)
        ctx.fb = fb
        ctx.save_for_backward(t, X)
        return u, du

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gu, gdu):
        fb = ctx.fb
        t, X = ctx.saved_tensors
        gu = torch.zeros(X.shape[0], device=X.device) if gu is None else gu.reshape(-1).float().contiguous()
        gdu = torch.zeros_like(X) if gdu is None else gdu.float().contiguous()
        g = torch.empty_like(fb.params)
        fb.solver.net_u_vjp(fb.params, t, X, gu, gdu, g)
        return (None, None, None) + fb._param_grads(g)


class _Loss(torch.autograd.Function):
    """FBSNN.loss_function's loss as a graph-connected scalar (the reference
    returns it with the graph built, DeepBSDE.py:278-279 / nd_BSPDE_case.py:378
    call loss.backward() on it).  Until a backward has been seen on the
    instance the forward is the forward-only native pass (dbsde_loss_grad
    without a gradient), so a caller that only evaluates or logs the loss pays
    no backward: it keeps the batch and a copy of the flat parameters (0.37 MB
    at the north star), and the backward runs dbsde_loss_grad on them -- the
    gradient of the weights the loss was evaluated at, as the reference's
    saved graph gives even if the parameters change in between.  Once a
    caller has called backward, later forwards compute loss and gradient in
    one fused pass and the backward only scales it (no second forward, no
    parameter copy).  The gradient is scaled by the incoming cotangent and
    split into the model parameters.  t, W and Xi are not differentiated; X
    and Y are returned detached (a loss built from Y gets no gradient through
    it: INTEGRATION.md)."""

    @staticmethod
    def forward(ctx, fb, t, W, Xi, *params):
        ctx.fb = fb
        if getattr(fb, "_loss_backward_seen", False):
            g = torch.empty_like(fb.params)
            out = fb._run(t, W, Xi, grad=g)
            ctx.grad = g
        else:
            out = fb._run(t, W, Xi)
            ctx.grad = None
            ctx.batch = (t, W, Xi)
            ctx.save_for_backward(fb.params.detach().clone())
        ctx.mark_non_differentiable(out["X"], out["Y"])
        return out["loss"][0].clone(), out["X"], out["Y"]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gl, gX, gY):
        fb = ctx.fb
        fb._loss_backward_seen = True
        if gl is None:
            return (None,) * (4 + len(fb._param_slices()))
        g = ctx.grad
        if g is None:
            (snap,) = ctx.saved_tensors
            t, W, Xi = ctx.batch
            g = torch.empty_like(snap)
            fb._run(t, W, Xi, grad=g, want=(), params=snap)
        return (None, None, None, None) + fb._param_grads(g * gl.float())


class FBSNN(ABC):
    """nd_BSPDE_case.py:126 / with_corr_high_dimension_pde.py:132 surface."""

    # reference behaviour switches (nd v2 defaults)
    clip_max_norm = 1.0          # nd_BSPDE_case.py:383 (DeepBSDE: none)
    schedule = "nd"              # Q1: "nd" (nd_BSPDE_case.py:364-368), "corr" (with_corr:406-409) or None
    skip_nonfinite = False       # heston_dnnpde.py:409-411 skips an iteration whose loss is NaN
    log_every = 100              # nd_BSPDE_case.py:395,402 (with_corr / hjb: 500)
    log_print = True             # nd / hjb print the logged iterations (with_corr's print is commented out)
    train_returns_time_logs = False   # with_corr...py:453, hjb_implement.py:450 return 4 values
    native_coefficients = True   # False: the subclass's own coefficient methods run (generic.py)
    generic_reason = None        # why they do (set by _select_problem)

    def __init__(self, Xi, T, M, N, D, Mm, layers, mode, activation, correlation_type="no_correlation",
                 device=None):
        self.device = torch.device(device) if device is not None else _default_device()
        self.T, self.M, self.N, self.D, self.Mm = T, M, N, D, Mm
        self.strike = self._default_strike()
        self.mode, self.activation = mode, activation
        self.layers = self._native_layers(list(layers))
        self.Xi = self._initial_state(Xi)
        spec = self._select_problem()
        self.spec = spec
        self.solver = NativeSolver(mode, self.layers, activation, spec, T, self.device)
        self.model = self._make_model(list(layers))
        self.params = networks.flatten_into(self.model, self.device)
        if self.params.numel() != self.solver.nparams:
            raise RuntimeError("native parameter layout does not match the module layout")
        # [grad | loss]: the native step writes both, one all-reduce sums both
        self._gradbuf = torch.zeros(self.params.numel() + 1, device=self.device)
        self.grad = self._gradbuf[:-1]
        self.training_loss = []
        self.iteration = []
        self.correlation_type = correlation_type
        self.correlation_matrix = self.generate_correlation_matrix(self.solver.nb)
        self._L = None if correlation_type == "no_correlation" else np.linalg.cholesky(self.correlation_matrix)
        if self._L is not None and spec.kind == "diag":
            self.solver.set_corr(self._L)       # device mode: L staged in LDS by the path kernel
        self.rank, self.world = _world()

    # ------------------------------------------------------------------ problem
    def _default_strike(self):
        return 1.0 * self.D          # nd_BSPDE_case.py:147

    def _native_layers(self, layers):
        return layers

    def _initial_state(self, Xi):
        return torch.as_tensor(np.asarray(Xi), dtype=torch.float32).to(self.device)

    def _make_model(self, layers):
        return networks.make_model(self.mode, layers, self.activation)

    def problem_spec(self):
        return None

    def _select_problem(self):
        """The coefficients the native step runs.  A subclass whose
        problem_spec() declares them, with every coefficient method it
        overrides agreeing with that declaration on probe inputs, runs them in
        the kernels (native_coefficients = True).  Any other subclass -- no
        spec, the reference's way of defining a problem (nd_BSPDE_case.py:
        458-500), or an override the inherited spec does not describe (e.g.
        class MyBSB(BlackScholesBarenblatt) with its own sigma_tf) -- runs its
        own methods through generic.py: its mu_tf / sigma_tf / phi_tf / g_tf /
        Dg_tf in torch, the network and its whole backward natively.  Returns
        the spec the native context is built with."""
        spec = self.problem_spec()
        why = None
        if spec is not None and not isinstance(spec, ProblemSpec):
            raise TypeError("problem_spec() must return a ProblemSpec or None")
        if spec is None:
            missing = [n for n in ("phi_tf", "g_tf") if generic.overridden(self, FBSNN, n) is None]
            if missing:
                raise NotImplementedError(f"{type(self).__name__} defines neither problem_spec() nor "
                                          f"{' / '.join(missing)} (the reference's abstract methods)")
            why = "no problem_spec()"
        else:
            bad = generic.coefficient_mismatches(self, FBSNN, spec, self.state_dim, self.T, self.Xi, self.device)
            if bad and spec.kind != "diag":
                raise NotImplementedError(f"{type(self).__name__} overrides {', '.join(bad)} of a {spec.kind!r} "
                                          "problem; only DIAG-shaped problems run user coefficient methods")
            if bad:
                why = f"{', '.join(bad)} differ from the inherited problem_spec()"
                warnings.warn(f"{type(self).__name__}: {why}; running the overridden methods (generic path)",
                              stacklevel=3)
        self.native_coefficients = why is None
        self.generic_reason = why
        if why is None:
            return spec
        generic.state_independence(self, self.state_dim, self.T, self.Xi, self.device)
        return ProblemSpec(q3=True)     # the context's network only; the coefficients run in generic.py

    def phi_tf(self, t, X, Y, Z):
        raise NotImplementedError

    def g_tf(self, X):
        raise NotImplementedError

    def mu_tf(self, t, X, Y, Z):
        return torch.zeros([X.shape[0], self.D], device=X.device)

    def sigma_tf(self, t, X, Y):
        return torch.diag_embed(torch.ones([X.shape[0], self.D], device=X.device))

    @property
    def state_dim(self):
        return self.layers[0] - 1

    # ------------------------------------------------------------------ correlation (with_corr:186-212)
    def generate_correlation_matrix(self, D):
        ct = getattr(self, "correlation_type", "no_correlation")
        if ct == "no_correlation":
            return np.eye(D)
        if ct == "random_correlation":
            return self._random_corr(D, False)
        if ct == "restricted_random_correlation":
            return self._random_corr(D, True)
        raise ValueError("Invalid correlation type")

    @staticmethod
    def _random_corr(D, positive):
        a = np.random.randn(D, D)
        if positive:
            a = np.abs(a)
        c = a @ a.T
        np.fill_diagonal(c, 1)          # before the normalisation, as the reference does (Q10)
        d = np.sqrt(np.diag(c))
        c = c / np.outer(d, d)
        eps = 1e-6
        while not np.all(np.linalg.eigvals(c) > 0):
            c += eps * np.eye(D)
            eps *= 2
        return c

    # ------------------------------------------------------------------ solver core
    def _host_minibatch(self, M=None):
        """DeepBSDE.py:247-262 / with_corr:316-353: the reference's numpy draw
        (the parity stream) in float64, cast to float32."""
        M = self.M if M is None else M
        N, nb, T = self.N, self.solver.nb, self.T
        Dt = np.zeros((M, N + 1, 1))
        DW = np.zeros((M, N + 1, nb))
        dt = T / N
        Dt[:, 1:, :] = dt
        dw = np.sqrt(dt) * np.random.normal(size=(M, N, nb))
        DW[:, 1:, :] = dw if self._L is None else np.einsum('ij,mnj->mni', self._L, dw)
        return np.cumsum(Dt, axis=1).astype(np.float32), np.cumsum(DW, axis=1).astype(np.float32)

    def fetch_minibatch(self):
        """Host numpy draws (the reference's stream), returned on the device."""
        t, W = self._host_minibatch()
        return torch.from_numpy(t).to(self.device), torch.from_numpy(W).to(self.device)

    def fetch_minibatch_device(self, seed=0, offset=0):
        """Device fetch_minibatch (Philox, correlated by L when set): t [M,N+1,1], W [M,N+1,nb]."""
        t, W = self.solver.brownian(self.M, self.N, seed=seed, offset=offset)
        return t.unsqueeze(-1), W

    def _xi_rows(self, Xi, M):
        Xi = torch.as_tensor(Xi, dtype=torch.float32).to(self.device).reshape(-1, self.state_dim).contiguous()
        if Xi.shape[0] not in (1, M):
            raise ValueError(f"Xi has {Xi.shape[0]} rows; expected 1 or {M}")
        return Xi

    def _local_xi(self, p0, ml, M):
        xi = self._xi_rows(self.Xi, M)
        return xi if xi.shape[0] == 1 else xi[p0:p0 + ml].contiguous()

    def _run(self, t, W, Xi, grad=None, want=("X", "Y"), loss=None, params=None):
        """One native loss(+grad) evaluation over the paths of t/W (at the
        model's parameters, or the flat vector `params`)."""
        M, N1 = t.shape[0], t.shape[1]
        N, Ds, nb = N1 - 1, self.state_dim, self.solver.nb
        Xi = self._xi_rows(Xi, M)
        if not self.native_coefficients:
            return generic.loss_grad(self, self.params if params is None else params, t, W, Xi, grad=grad,
                                     want=want, loss_out=loss)
        out = {"loss": torch.empty(1, device=self.device) if loss is None else loss}
        if "X" in want:
            out["X"] = torch.empty((M, N1, Ds), device=self.device)
        if "Y" in want:
            out["Y"] = torch.empty((M, N1, 1), device=self.device)
        if "Z" in want:
            out["Z"] = torch.empty((M, N1, Ds), device=self.device)
        t = torch.as_tensor(t, dtype=torch.float32).to(self.device)
        W = torch.as_tensor(W, dtype=torch.float32).to(self.device)
        self.solver.loss_grad(self.params if params is None else params, M, N, Xi, t=t.reshape(M, N1).contiguous(),
                              W=W.reshape(M, N1, nb).contiguous(), grad=grad, loss=out["loss"],
                              X=out.get("X"), Y=out.get("Y"), Z=out.get("Z"))
        return out

    def net_u(self, t, X):
        """DeepBSDE.py:189-194: (u [R,1], Du [R,D]) at the given points.  With
        grad mode on, (u, Du) are connected to the model parameters as in the
        reference (nd_BSPDE_case.py:191-221, create_graph=True): a backward
        through them runs the native VJP (dbsde_net_u_vjp) and accumulates
        into each parameter's .grad.  The points are not differentiated."""
        X = torch.as_tensor(X, dtype=torch.float32).to(self.device)
        if X.dim() == 1:
            X = X.unsqueeze(-1)
        t = torch.as_tensor(t, dtype=torch.float32).to(self.device).reshape(-1).contiguous()
        X = X.detach().reshape(-1, self.state_dim).contiguous()
        params = [p for _, p in self.model.named_parameters()]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _NetU.apply(self, t, X, *params)
        u = torch.empty((X.shape[0], 1), device=self.device)
        du = torch.empty_like(X)
        self.solver.net_u(self.params, t, X, u, du)
        return u, du

    def _param_grads(self, g):
        """A flat gradient split into named_parameters() order; None for a
        parameter no output depends on (NAIS-Net's input_layers[K]),
        whose .grad torch autograd leaves None as well."""
        if getattr(self, "_pused", None) is None:
            used = self.solver.used_mask
            self._pused = [bool(used[o:o + n].any()) for o, n, _ in self._param_slices()]
        return tuple(g[o:o + n].view(shape) if u else None
                     for (o, n, shape), u in zip(self._param_slices(), self._pused))

    def _param_slices(self):
        """(offset, numel, shape) of every model parameter in the flat vector, in
        named_parameters() order (the flat vector is in state_dict order,
        networks.bind)."""
        if getattr(self, "_pslices", None) is None:
            off, where = 0, {}
            for name, p in self.model.state_dict().items():
                where[name] = (off, p.numel(), p.shape)
                off += p.numel()
            self._pslices = [where[name] for name, _ in self.model.named_parameters()]
        return self._pslices

    def Dg_tf(self, X):
        """DeepBSDE.py:196-200 (torch autograd of the problem's g_tf)."""
        X = X.detach().requires_grad_(True)
        g = self.g_tf(X)
        return torch.autograd.grad(g, X, torch.ones_like(g))[0]

    def loss_function(self, t, W, Xi):
        """nd_BSPDE_case.py:237-281 -> (loss, X, Y, Y[0,0,0]).  With grad mode
        on and the model's parameters requiring grad, the loss is connected to
        them like the reference's: loss.backward() accumulates the native
        gradient (dbsde_loss_grad, run by the backward) into each parameter's
        .grad.  X and Y are returned detached."""
        params = [p for _, p in self.model.named_parameters()]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            loss, X, Y = _Loss.apply(self, t, W, Xi, *params)
            return loss, X, Y, Y[0, 0, 0]
        out = self._run(t, W, Xi)
        Y = out["Y"]
        return out["loss"][0], out["X"], Y, Y[0, 0, 0]

    # ------------------------------------------------------------------ training
    def _schedule_n(self, it):
        if self.schedule == "nd" and self.Mm is not None:
            if 4000 <= it < 20000:
                self.N = int(np.ceil(self.Mm ** (int(it / 4000) + 1)))
            elif it < 4000:
                self.N = int(np.ceil(self.Mm))
        elif self.schedule == "corr":
            if 4000 <= it < 20000:
                self.N = int(np.ceil((self.N ** (1 / 5)) ** (int(it / 4000) + 1)))
            elif it < 4000:
                self.N = int(np.ceil(self.N ** (1 / 5)))

    def _local_slice(self, M):
        if self.world == 1:
            return 0, M
        if M % self.world:
            raise ValueError(f"M={M} is not divisible by the world size {self.world}")
        if self.state_dim == 1 and self.spec.q3:
            # the reference's D == 1 Y-tilde term sums sigma*dW over ALL
            # M paths, which a path-sharded rank cannot see
            raise ValueError("the D == 1 squeeze-broadcast problems (q3) cannot be sharded over ranks")
        m = M // self.world
        return self.rank * m, m

    def _check_optimizer(self, optimizer_type):
        if optimizer_type not in OPTIMIZER_NAMES:
            raise ValueError(f"Optimizer type '{optimizer_type}' is not recognized.")

    def new_optimizer_state(self, optimizer_type="Adam", learning_rate=None):
        """A fresh optimizer (the reference builds one per train() call, Q11)."""
        self._check_optimizer(optimizer_type)
        if optimizer_type == "LBFGS":
            return self._lbfgs_state(learning_rate)
        # "dstep": the update count lives on the device (dbsde_optim.step_state),
        # so an update skipped for a non-finite loss does not advance Adam's bias
        # corrections or ASGD's eta / mu (heston_dnnpde.py:409-411 skips before
        # optimizer.step()); "calls" counts the launches (ping-pong slot)
        return {"kind": optimizer_type, "lr": learning_rate, "m": torch.zeros_like(self.params),
                "v": torch.zeros_like(self.params), "dstep": torch.zeros(2, dtype=torch.float64, device=self.device),
                "calls": 0}

    def _opt_kwargs(self, opt, learning_rate=None, skip_loss=None):
        """The optimizer_step keywords of the next update of `opt` (advances its
        launch count: the device step counter's ping-pong slot)."""
        kind = opt["kind"]
        if kind == "LBFGS":
            raise ValueError("LBFGS steps need a closure (FBSNN._lbfgs_step)")
        lr = opt["lr"] if learning_rate is None else learning_rate
        kw = OPT_DEFAULTS[kind]
        parity = opt["calls"] & 1
        opt["calls"] += 1
        return dict(kind=kind, lr=lr, betas=kw.get("betas", (0.9, 0.999)), eps=kw.get("eps", 1e-8),
                    weight_decay=kw["weight_decay"], max_norm=self.clip_max_norm or 0.0, step=opt["calls"],
                    alpha=kw.get("alpha", 0.99) if kind == "RMSprop" else 0.99, rho=kw.get("rho", 0.9),
                    lr_decay=kw.get("lr_decay", 0.0), lambd=kw.get("lambd", 1e-4), skip_nonfinite_loss=skip_loss,
                    step_state=opt["dstep"], step_parity=parity)

    def _update(self, opt, learning_rate=None, skip_loss=None):
        """clip_grad_norm_ (not for LBFGS) + optimizer.step() on the device."""
        self.solver.optimizer_step(self.params, self.grad, opt["m"], opt["v"],
                                   **self._opt_kwargs(opt, learning_rate, skip_loss))

    def optimizer_steps_taken(self, opt):
        """Updates the device has applied (skipped ones excluded); syncs."""
        return int(opt["dstep"][opt["calls"] & 1].item())

    # ------------------------------------------------------------------ L-BFGS
    def _lbfgs_state(self, lr):
        """torch.optim.LBFGS(params, lr) with its defaults (nd_BSPDE_case.py:347-348):
        max_iter 20, max_eval 25, tolerance_grad 1e-7, tolerance_change 1e-9,
        history_size 100, no line search.  The history lives in two device
        matrices of history_size + 1 rows (one scratch row for the candidate
        pair before torch's ys > 1e-10 test)."""
        n = self.params.numel()
        H = 100
        z = lambda *shape: torch.zeros(*shape, device=self.device)   # noqa: E731
        return {"kind": "LBFGS", "lr": 1.0 if lr is None else lr, "max_iter": 20, "max_eval": 25,
                "tolerance_grad": 1e-7, "tolerance_change": 1e-9, "history_size": H,
                "S": z(H + 1, n), "Y": z(H + 1, n), "slots": [], "ro": [], "free": list(range(H + 1)),
                "d": z(n), "prev_g": z(n), "t": None, "H_diag": 1.0, "prev_loss": None, "n_iter": 0,
                "func_evals": 0}

    def _lbfgs_step(self, st, closure):
        """torch.optim.LBFGS.step(closure) (torch 2.10, line_search_fn=None)
        restated: the same control flow and fp32 scalars, every vector
        operation on the device (dbsde_vec_reduce / dbsde_vec_axpby /
        dbsde_lbfgs_direction).  closure() re-runs the native loss and gradient
        into self.grad on the same batch and returns the loss as a float.
        Returns the loss of the first evaluation (torch's orig_loss)."""
        sv, g, d, f32 = self.solver, self.grad, st["d"], np.float32
        lr, tol_grad, tol_change = st["lr"], st["tolerance_grad"], st["tolerance_change"]
        orig_loss = closure()
        loss = orig_loss
        current_evals = 1
        st["func_evals"] += 1
        if sv.vec_reduce("amax", g) <= tol_grad:
            return orig_loss
        t = st["t"]
        n_iter = 0
        while n_iter < st["max_iter"]:
            n_iter += 1
            st["n_iter"] += 1
            if st["n_iter"] == 1:
                sv.vec_axpby(d, g, -1.0)                                   # d = -g
                st["slots"], st["ro"], st["H_diag"] = [], [], 1.0
                st["free"] = list(range(st["history_size"] + 1))
            else:
                c = st["free"][0]
                y, s = st["Y"][c], st["S"][c]
                sv.vec_axpby(y, g, 1.0, st["prev_g"], -1.0)                # y = g - prev_g
                sv.vec_axpby(s, d, float(f32(t)))                          # s = d * t
                ys = f32(sv.vec_reduce("dot", y, s))
                if ys > 1e-10:
                    if len(st["slots"]) == st["history_size"]:
                        st["free"].append(st["slots"].pop(0))
                        st["ro"].pop(0)
                    st["free"].remove(c)
                    st["slots"].append(c)
                    st["ro"].append(float(f32(1.0) / ys))
                    st["H_diag"] = float(ys / f32(sv.vec_reduce("dot", y, y)))
                sv.lbfgs_direction(g, st["S"], st["Y"], st["slots"], st["ro"], st["H_diag"], d)
            sv.vec_axpby(st["prev_g"], g, 1.0)
            prev_loss = loss
            if st["n_iter"] == 1:
                inv = f32(1.0) / f32(sv.vec_reduce("asum", g))
                t = float(f32(inv * f32(lr))) if inv < 1.0 else 1.0 * lr
            else:
                t = lr
            gtd = f32(sv.vec_reduce("dot", g, d))
            if gtd > -tol_change:
                break
            ls_func_evals = 0
            sv.vec_axpby(self.params, d, float(f32(t)), self.params, 1.0)   # _add_grad(t, d)
            opt_cond = False
            if n_iter != st["max_iter"]:
                loss = closure()
                opt_cond = sv.vec_reduce("amax", g) <= tol_grad
                ls_func_evals = 1
            current_evals += ls_func_evals
            st["func_evals"] += ls_func_evals
            if n_iter == st["max_iter"] or current_evals >= st["max_eval"] or opt_cond:
                break
            if f32(sv.vec_reduce("amax", d)) * abs(f32(t)) <= tol_change:
                break
            if abs(loss - prev_loss) < tol_change:
                break
        st["t"] = t
        st["prev_loss"] = prev_loss
        return orig_loss

    def _reduce(self):
        if self.world > 1:
            dist.all_reduce(self._gradbuf)     # RCCL over xGMI: [grad | loss], ~0.37 MB
        return self._gradbuf[-1:]

    def _closure(self, t, W, p0, ml, M):
        """The reference's LBFGS closure (nd_BSPDE_case.py:357-361): loss and
        gradient again on the same batch; returns the (all-reduced) loss."""
        self._run(t[p0:p0 + ml], W[p0:p0 + ml], self._local_xi(p0, ml, M), grad=self.grad, want=(),
                  loss=self._gradbuf[-1:])
        return float(self._reduce().item())

    def train_step(self, t, W, opt_state, optimizer_type=None, learning_rate=None, want_state=False):
        """loss/grad on the local shard of a global minibatch (t, W: host numpy
        or device tensors of all M paths) -> all-reduce -> clip -> optimizer
        step.  Returns (device loss, outputs of the local shard)."""
        M = t.shape[0]
        p0, ml = self._local_slice(M)
        out = self._run(t[p0:p0 + ml], W[p0:p0 + ml], self._local_xi(p0, ml, M), grad=self.grad,
                        want=("X", "Y") if want_state else (), loss=self._gradbuf[-1:])
        loss = self._reduce()
        if opt_state["kind"] == "LBFGS":
            loss = loss.clone()
            self._lbfgs_step(opt_state, lambda: self._closure(t, W, p0, ml, M))
            return loss, out
        self._update(opt_state, learning_rate, skip_loss=loss if self.skip_nonfinite else None)
        return loss, out

    def _device_xi(self, p0, ml):
        """The persistent device copy of this shard's Xi that device-mode batches
        (and their prefetch, which matches on the pointer) read.  It is
        refreshed whenever self.Xi is replaced or modified in place (tensor
        version counter), so a changed Xi is never served from a stale copy."""
        src = self.Xi
        key = (p0, ml, self.M, id(src), getattr(src, "_version", None))
        if getattr(self, "_xi_dev_key", None) != key:
            xi = self._local_xi(p0, ml, self.M)
            if getattr(self, "_xi_dev", None) is not None and self._xi_dev.shape == xi.shape:
                # the pending prefetch read the old values: drop it before rewriting
                self.solver.prefetch_drop()
                self._xi_dev.copy_(xi)
            else:
                self._xi_dev = xi.clone()
            self._xi_dev_src = src          # keeps id(src) from being reused while cached
            self._xi_dev_key = key
        return self._xi_dev

    def device_step(self, opt_state, learning_rate=None, seed=0, optimizer_type=None, next_seed=None):
        """Throughput-mode iteration: Brownian increments drawn on the device
        (Philox keyed by global path index, correlated by L when set),
        loss+grad, all-reduce, clip + optimizer.  No host synchronisation;
        returns the device loss.  next_seed: the seed of the following
        iteration, whose rollout is then prefetched to overlap this one
        (dbsde_prefetch); the numbers are the same either way."""
        if self._L is not None and self.spec.kind != "diag":
            raise NotImplementedError("device-mode correlated increments are implemented for diagonal problems")
        p0, ml = self._local_slice(self.M)
        xi = self._device_xi(p0, ml)
        lbfgs = opt_state["kind"] == "LBFGS"
        if not self.native_coefficients:
            # user coefficient methods (generic.py): the same device Philox
            # increments, exported, then the generic loss and native backward
            t, W = self.solver.brownian(ml, self.N, seed=seed, path0=p0)

            def closure():
                self._run(t, W, xi, grad=self.grad, want=(), loss=self._gradbuf[-1:])
                return self._reduce()
            loss = closure()
            if lbfgs:
                loss = loss.clone()
                self._lbfgs_step(opt_state, lambda: float(closure().item()))
                return loss
            self._update(opt_state, learning_rate, skip_loss=loss if self.skip_nonfinite else None)
            return loss
        if next_seed is not None and not lbfgs:
            self.solver.prefetch(ml, self.N, xi, seed=next_seed, path0=p0)
        if self.world == 1 and not lbfgs:
            # one process: loss, gradient and update in one native call (the
            # update folds into the gradient finalize when it can)
            self.solver.train_step(self.params, ml, self.N, xi, self.grad, opt_state["m"], opt_state["v"],
                                   self._opt_kwargs(opt_state, learning_rate,
                                                    self._gradbuf[-1:] if self.skip_nonfinite else None),
                                   seed=seed, path0=p0, loss=self._gradbuf[-1:])
            return self._gradbuf[-1:]
        self.solver.loss_grad(self.params, ml, self.N, xi, seed=seed, path0=p0,
                              grad=self.grad, loss=self._gradbuf[-1:])
        loss = self._reduce()
        if lbfgs:
            def closure():
                self.solver.loss_grad(self.params, ml, self.N, xi, seed=seed, path0=p0, grad=self.grad,
                                      loss=self._gradbuf[-1:])
                return float(self._reduce().item())
            loss = loss.clone()
            self._lbfgs_step(opt_state, closure)
            return loss
        self._update(opt_state, learning_rate, skip_loss=loss if self.skip_nonfinite else None)
        return loss

    def train_device(self, N_Iter, learning_rate, seed=0, optimizer_type="Adam"):
        """train() with device-generated Brownian increments (no numpy stream,
        no per-iteration host sync except every log_every iterations).  Like
        the reference's NaN skip (heston_dnnpde.py:409-411), non-finite losses
        are left out of the logged window means."""
        previous_it = self.iteration[-1] if self.iteration else 0
        opt_state = self.new_optimizer_state(optimizer_type, learning_rate)
        losses = []
        for it in range(previous_it, previous_it + N_Iter):
            self._schedule_n(it)
            nxt = (seed << 20) + it + 1 if it + 1 < previous_it + N_Iter else None
            losses.append(self.device_step(opt_state, learning_rate, seed=(seed << 20) + it, next_seed=nxt).clone())
            if it % self.log_every == 0:
                window = torch.cat(losses)
                if self.skip_nonfinite:
                    window = window[torch.isfinite(window)]
                self.training_loss.append(float(window.mean()) if window.numel() else float("nan"))
                losses = []
                self.iteration.append(it)
        return np.stack((self.iteration, self.training_loss))

    def _record_y0(self, out):
        pass

    def _train_graph(self):
        return np.stack((self.iteration, self.training_loss))

    def train(self, N_Iter, learning_rate, optimizer_type='Adam'):
        """nd_BSPDE_case.py:316-410 -> (graph, min_loss, min_loss_state); the
        with_corr / hjb classes (train_returns_time_logs) log every 500
        iterations and also return time_logs (with_corr...py:355-453,
        hjb_implement.py:394-450).  LBFGS runs optimizer.step(closure) with the
        native loss as the closure and no clipping, as the reference does."""
        opt_state = self.new_optimizer_state(optimizer_type, learning_rate)   # fresh per call (Q11)
        lbfgs = optimizer_type == "LBFGS"
        loss_temp = []
        previous_it = self.iteration[-1] if self.iteration else 0
        start_time = time.time()
        cumulative_time, time_logs = 0.0, []
        min_loss, min_loss_state = float('inf'), None
        for it in range(previous_it, previous_it + N_Iter):
            self._schedule_n(it)
            t_np, W_np = self._host_minibatch()       # the global batch; each rank uploads its slice
            M = t_np.shape[0]
            p0, ml = self._local_slice(M)
            out = self._run(t_np[p0:p0 + ml], W_np[p0:p0 + ml], self._local_xi(p0, ml, M), grad=self.grad,
                            want=("X", "Y"), loss=self._gradbuf[-1:])
            loss = float(self._reduce().item())
            if self.skip_nonfinite and not np.isfinite(loss):
                print(f"NaN loss detected at iteration {it}. Skipping this iteration")
                continue
            if lbfgs:
                self._lbfgs_step(opt_state, lambda: self._closure(t_np, W_np, p0, ml, M))
            else:
                self._update(opt_state, learning_rate)
            loss_temp.append(loss)
            if loss < min_loss:
                min_loss = loss
                min_loss_state = (out["X"].clone(), out["Y"].clone())
            if it % self.log_every == 0:
                elapsed = time.time() - start_time
                cumulative_time += elapsed
                time_logs.append(cumulative_time)
                if self.rank == 0 and self.log_print:
                    y0 = float(out["Y"][0, 0, 0])
                    print(f'It: {it}, Loss: {loss:.3e}, Y0: {y0:.3f}, Time: {elapsed:.2f}, '
                          f'Learning Rate: {learning_rate:.3e}')
                start_time = time.time()
                self.training_loss.append(float(np.mean(loss_temp)))
                loss_temp = []
                self.iteration.append(it)
                self._record_y0(out)
        if self.train_returns_time_logs:
            return self._train_graph(), min_loss, min_loss_state, time_logs
        return self._train_graph(), min_loss, min_loss_state

    # ------------------------------------------------------------------ inference
    def predict(self, Xi_star, t_star, W_star):
        """nd_BSPDE_case.py:412-443 (sets self.M to the batch size)."""
        Xi_star = torch.as_tensor(np.asarray(Xi_star) if not isinstance(Xi_star, torch.Tensor) else Xi_star,
                                  dtype=torch.float32).to(self.device).reshape(-1, self.state_dim)
        t_star = torch.as_tensor(t_star, dtype=torch.float32).to(self.device)
        W_star = torch.as_tensor(W_star, dtype=torch.float32).to(self.device)
        bs = max(Xi_star.shape[0], t_star.shape[0], W_star.shape[0])
        self.M = bs
        if t_star.shape[0] == 1:
            t_star = t_star.repeat(bs, 1, 1)
        if W_star.shape[0] == 1:
            W_star = W_star.repeat(bs, 1, 1)
        out = self._run(t_star, W_star, Xi_star)
        return out["X"], out["Y"]

    # ------------------------------------------------------------------ checkpoints
    def save_model(self, file_name):
        torch.save({'model_state_dict': self.model.state_dict(), 'training_loss': self.training_loss,
                    'iteration': self.iteration}, file_name)

    def load_model(self, file_name):
        """nd_BSPDE_case.py:452-456.  The reference stores training_loss as numpy
        float64 scalars; they are allow-listed for the weights-only loader (no
        arbitrary unpickling) and converted to Python floats."""
        safe = [np.dtype, type(np.dtype(np.float64)), type(np.dtype(np.int64))]
        try:
            safe.append(np._core.multiarray.scalar)
        except AttributeError:  # numpy < 2
            safe.append(np.core.multiarray.scalar)
        with torch.serialization.safe_globals(safe):
            ck = torch.load(file_name, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck['model_state_dict'])
        self.training_loss = [float(v) for v in ck['training_loss']]
        self.iteration = [int(v) for v in ck['iteration']]


class PredictionGenerator:
    """nd_BSPDE_case.py:543-584: num_samples batches of predictions from the
    reference's numpy stream seeded with 42, concatenated over paths."""

    def __init__(self, model, Xi, num_samples):
        self.model = model
        self.Xi = Xi
        self.num_samples = num_samples

    def generate_predictions(self):
        np.random.seed(42)
        ts, Xs, Ys = [], [], []
        W_test = None
        for _ in range(self.num_samples):
            t_i, W_i = self.model.fetch_minibatch()
            X_i, Y_i = self.model.predict(self.Xi, t_i, W_i)[:2]
            if W_test is None:
                W_test = W_i
            ts.append(t_i.cpu().numpy())
            Xs.append(X_i.cpu().numpy())
            Ys.append(Y_i.cpu().numpy())
        return np.concatenate(ts, 0), W_test, np.concatenate(Xs, 0), np.concatenate(Ys, 0)


__all__ = ["FBSNN", "PredictionGenerator", "ProblemSpec", "OPTIMIZER_NAMES", "NATIVE_OPTIMIZERS", "OPT_DEFAULTS"]
