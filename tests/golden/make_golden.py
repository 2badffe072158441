"""Generate the golden parity vectors by running the REFERENCE itself.

Run in the build container only (it reads /root/reference, which the GPU box
does not have):   python tests/golden/make_golden.py
The outputs (tests/golden/*.npz) are data -- inputs and the reference's
outputs -- and are what the oracle and the HIP path are checked against.

Each case seeds torch and numpy, constructs the reference problem class
(so the reference's own init runs), draws the reference's own minibatch,
runs the reference loss_function and loss.backward(), and stores
  params (flat, state_dict order), t, W, Xi, loss, X, Y, Z (via the
  reference net_u on the reference X), grad (flat) and used-mask.
Training cases additionally run the reference train() and store the final
parameters.  seaborn is not installed here; the reference imports it only for
plotting, so an empty stub module is registered.
"""
from __future__ import annotations

import contextlib
import importlib.util
import io
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _load(fname, modname):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, fname))
    mod = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()):
        spec.loader.exec_module(mod)
    return mod


def _setup():
    import matplotlib
    matplotlib.use("Agg")
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
    sys.path.insert(0, REF)
    mods = dict(
        deep=_load("DeepBSDE.py", "ref_DeepBSDE"),
        nd=_load("nd_BSPDE_case.py", "ref_nd"),
        corr=_load("with_corr_high_dimension_pde.py", "ref_corr"),
        hjb=_load("hjb_implement.py", "ref_hjb"),
        oned=_load("1d_BSPDE_case.py", "ref_1d"),
        heston=_load("heston_dnnpde.py", "ref_heston"),
    )
    import torch
    torch.autograd.set_detect_anomaly(False)   # DeepBSDE.py:11 turns it on (Q8); speed only
    torch.set_num_threads(1)                  # deterministic reductions
    return mods


def _flat(sd):
    import torch
    return torch.cat([p.detach().reshape(-1) for p in sd.values()]).numpy().astype(np.float32)


def _grads(model):
    params = dict(model.named_parameters())
    g, m = [], []
    for name, p in model.state_dict().items():
        q = params[name]
        if q.grad is None:
            g.append(np.zeros(q.numel(), np.float32))
            m.append(np.zeros(q.numel(), bool))
        else:
            g.append(q.grad.detach().reshape(-1).numpy())
            m.append(np.ones(q.numel(), bool))
    return np.concatenate(g), np.concatenate(m)


def _run_case(obj, M, N, D, full_z=True):
    """Reference minibatch + loss + backward on `obj` (a reference FBSNN)."""
    import torch
    with contextlib.redirect_stdout(io.StringIO()):
        t, W = obj.fetch_minibatch()
        obj.model.zero_grad(set_to_none=True)
        out = obj.loss_function(t, W, obj.Xi)
        loss, X, Y = out[0], out[1], out[2]
        loss.backward()
        g, used = _grads(obj.model)
        Zs = []
        if full_z:
            for n in range(N + 1):
                Xn = X[:, n, :].detach().clone().requires_grad_(True)
                _, zn = obj.net_u(t[:, n, :], Xn)
                Zs.append(zn.detach())
    res = dict(t=t.numpy(), W=W.numpy(), loss=np.float64(loss.item()),
               X=X.detach().numpy(), Y=Y.detach().numpy(), grad=g, used=used)
    if full_z:
        res["Z"] = torch.stack(Zs, 1).numpy()
    return res


def small_cases(mods):
    """G1/G3: small shapes over archs x activations x problems (+ quirks)."""
    import torch
    T = 1.0
    cases = []
    D4 = 4
    L4 = [D4 + 1, 16, 16, 16, 16, 1]
    xi_bsb = np.array([1.0, 0.5] * (D4 // 2))[None, :]
    for mode in ["NAIS-Net", "Resnet", "FC"]:
        for act in ["Sine", "ReLU"]:
            cases.append((f"deep_bsb_{mode}_{act}", "deep", "BlackScholesBarenblatt", "bsb", mode, act,
                          L4, xi_bsb, 8, 5, {}))
    for mode in ["Naisnet", "FC"]:
        for act in ["Sine", "ReLU", "Tanh"]:
            cases.append((f"nd_call_{mode}_{act}", "nd", "CallOption", "call", mode, act,
                          L4, np.ones((1, D4)), 8, 5, {"Mm": 5.0}))
    cases.append(("nd_call_Naisnet_Sine_len4", "nd", "CallOption", "call", "Naisnet", "Sine",
                  [D4 + 1, 16, 16, 1], np.ones((1, D4)), 8, 5, {"Mm": 5.0}))
    cases.append(("nd_call_Naisnet_Tanh_len5", "nd", "CallOption", "call", "Naisnet", "Tanh",
                  [D4 + 1, 16, 16, 16, 1], np.ones((1, D4)), 8, 5, {"Mm": 5.0}))
    cases.append(("corr_basket_Naisnet_ReLU", "corr", "CallOption", "basket", "Naisnet", "ReLU",
                  L4, np.ones((1, D4)), 8, 5, {"Mm": 5.0, "correlation_type": "random_correlation"}))
    cases.append(("corr_basket_Naisnet_Sine_restricted", "corr", "CallOption", "basket", "Naisnet", "Sine",
                  L4, np.ones((1, D4)), 8, 5,
                  {"Mm": 5.0, "correlation_type": "restricted_random_correlation"}))
    cases.append(("corr_bspdetest_Naisnet_Sine", "corr", "BSPDETestCase", "bspde_test", "Naisnet", "Sine",
                  L4, xi_bsb, 8, 5, {"Mm": 5.0}))
    for mode, act in [("FC", "Sine"), ("Naisnet", "ReLU")]:
        cases.append((f"hjb_{mode}_{act}", "hjb", "HamiltonJacobiBellman", "hjb", mode, act,
                      L4, np.zeros((1, D4)), 8, 5, {}))
    for mode, act, M in [("FC", "Sine", 4), ("Naisnet", "Tanh", 6), ("FC", "ReLU", 1)]:
        cases.append((f"oned_call_{mode}_{act}_M{M}", "oned", "CallOption", "call1d", mode, act,
                      [2, 16, 16, 16, 16, 1], np.array([[1.0]]), M, 5, {"Mm": 5.0}))

    for seed, (name, modkey, cls, prob, mode, act, layers, Xi, M, N, kw) in enumerate(cases):
        torch.manual_seed(seed)
        np.random.seed(seed)
        C = getattr(mods[modkey], cls)
        D = layers[0] - 1
        with contextlib.redirect_stdout(io.StringIO()):
            if modkey == "deep":
                obj = C(Xi, T, M, N, D, layers, mode, act)
            elif modkey == "hjb":
                obj = C(Xi, T, M, N, D, layers, mode, act)
            elif modkey == "corr":
                obj = C(Xi, T, M, N, D, kw["Mm"], layers, mode, act,
                        kw.get("correlation_type", "no_correlation"))
            else:
                obj = C(Xi, T, M, N, D, kw["Mm"], layers, mode, act)
        params = _flat(obj.model.state_dict())
        res = _run_case(obj, M, N, D)
        extra = {}
        if modkey in ("corr", "hjb"):
            extra["corr"] = np.asarray(obj.correlation_matrix, np.float64)
        np.savez_compressed(os.path.join(OUT, f"g1_{name}.npz"), name=name, problem=prob, mode=mode,
                            activation=act, layers=np.array(layers), Xi=Xi.astype(np.float32),
                            M=M, N=N, T=T, seed=seed, params=params, **res, **extra)
        print(f"{name:42s} loss={res['loss']:.6e}")


def _save_case(name, prob, mode, act, layers, Xi, M, N, seed, params, res, **extra):
    np.savez_compressed(os.path.join(OUT, f"g1_{name}.npz"), name=name, problem=prob, mode=mode, activation=act,
                        layers=np.array(layers), Xi=np.asarray(Xi, np.float32), M=M, N=N, T=1.0, seed=seed,
                        params=params, **res, **extra)
    print(f"{name:42s} loss={res['loss']:.6e}", flush=True)


def wide_cases(mods):
    """Round 2: the north-star width (fused T=7 kernels) for ReLU / Tanh, the
    Q4 not-taken branch, config 3 (basket D=100 + Cholesky L, Naisnet-ReLU) and
    config 4 (HJB FC-Sine [101,256x4,1], N=20) at small M."""
    import torch
    D = 100
    L110 = [D + 1] + 4 * [110] + [1]
    xi_bsb = np.array([1.0, 0.5] * (D // 2))[None, :]
    specs = [
        ("w110_deep_bsb_NAIS-Net_ReLU", "deep", "BlackScholesBarenblatt", "bsb", "NAIS-Net", "ReLU", L110, xi_bsb,
         16, 5, {}),
        ("w110_nd_call_Naisnet_Tanh", "nd", "CallOption", "call", "Naisnet", "Tanh", L110, np.ones((1, D)), 16, 5,
         {"Mm": 5.0}),
        ("w110_corr_basket_Naisnet_ReLU", "corr", "CallOption", "basket", "Naisnet", "ReLU", L110, np.ones((1, D)),
         16, 5, {"Mm": 5.0, "correlation_type": "random_correlation"}),
        ("w256_hjb_FC_Sine_N20", "hjb", "HamiltonJacobiBellman", "hjb", "FC", "Sine", [D + 1] + 4 * [256] + [1],
         np.zeros((1, D)), 16, 20, {}),
        ("q4off_deep_bsb_NAIS-Net_Sine", "deep", "BlackScholesBarenblatt", "bsb", "NAIS-Net", "Sine",
         [5, 16, 16, 16, 16, 1], np.array([1.0, 0.5] * 2)[None, :], 8, 5, {"scale_hidden": 0.05}),
        ("q4off_nd_call_Naisnet_Tanh", "nd", "CallOption", "call", "Naisnet", "Tanh", [5, 16, 16, 16, 1],
         np.ones((1, 4)), 8, 5, {"Mm": 5.0, "scale_hidden": 0.05}),
    ]
    for k, (name, modkey, cls, prob, mode, act, layers, Xi, M, N, kw) in enumerate(specs):
        seed = 300 + k
        torch.manual_seed(seed)
        np.random.seed(seed)
        C = getattr(mods[modkey], cls)
        Dd = layers[0] - 1
        with contextlib.redirect_stdout(io.StringIO()):
            if modkey in ("deep", "hjb"):
                obj = C(Xi, 1.0, M, N, Dd, layers, mode, act)
            elif modkey == "corr":
                obj = C(Xi, 1.0, M, N, Dd, kw["Mm"], layers, mode, act, kw.get("correlation_type", "no_correlation"))
            else:
                obj = C(Xi, 1.0, M, N, Dd, kw["Mm"], layers, mode, act)
        extra = {}
        if "scale_hidden" in kw:        # drive |W^T W|_F below 0.98: the Q4 branch is not taken
            with torch.no_grad():
                norms = []
                for name_, prm in obj.model.named_parameters():
                    hidden = name_.startswith("hidden_layers.") or (name_.startswith("layer") and "_input" not in name_
                                                                    and name_.split(".")[0] not in ("layer1",)
                                                                    and name_.split(".")[0] != f"layer{len(layers) - 1}")
                    if hidden and name_.endswith("weight"):
                        prm.mul_(kw["scale_hidden"])
                        norms.append(float(torch.norm(prm.t() @ prm)))
            assert norms and max(norms) < 0.98, norms
            extra["rtr_norms"] = np.array(norms)
        params = _flat(obj.model.state_dict())
        res = _run_case(obj, M, N, Dd)
        if modkey in ("corr", "hjb"):
            extra["corr"] = np.asarray(obj.correlation_matrix, np.float64)
        _save_case(name, prob, mode, act, layers, Xi, M, N, seed, params, res, **extra)


def _heston_run(obj, M, N):
    """Reference Heston minibatch + loss + backward; Z = (dU/dS, dU/dv) from its net_u."""
    import torch
    with contextlib.redirect_stdout(io.StringIO()):
        t, W = obj.fetch_minibatch()
        obj.model.zero_grad(set_to_none=True)
        loss, X, Y, _ = obj.loss_function(t, W, obj.Xi)
        loss.backward()
        g, used = _grads(obj.model)
        Zs = []
        for n in range(N + 1):
            Xn = X[:, n, :].detach().clone().requires_grad_(True)
            _, zs, zv = obj.net_u(t[:, n, :], Xn)
            Zs.append(torch.cat([zs, zv], 1).detach())
    return dict(t=t.numpy(), W=W.numpy(), loss=np.float64(loss.item()), X=X.detach().numpy(),
                Y=Y.detach().numpy(), grad=g, used=used, Z=torch.stack(Zs, 1).numpy())


def heston_cases(mods):
    """Config 5 at the reference's only scope, one asset (heston_dnnpde.py:519-659):
    loss/grad fixtures for both payoffs and both modes, and a 10-iteration train()."""
    import torch
    H = mods["heston"].HestonFBSNN
    layers = [2, 16, 16, 16, 16, 1]
    hp = dict(kappa=2.0, theta=0.2, sigma=0.3, rho=0.8, v0=0.2)
    specs = [("heston_Naisnet_Sine", "Naisnet", "Sine", "discontinuous", 8, 5),
             ("heston_Naisnet_Tanh_continuous", "Naisnet", "Tanh", "continuous", 8, 5),
             ("heston_FC_Sine", "FC", "Sine", "discontinuous", 6, 4)]
    for k, (name, mode, act, payoff, M, N) in enumerate(specs):
        seed = 400 + k
        torch.manual_seed(seed)
        np.random.seed(seed)
        Xi = np.array([[1.0]])
        with contextlib.redirect_stdout(io.StringIO()):
            obj = H(Xi, 1.0, M, N, 1, 5.0, layers, mode, act, payoff_type=payoff, **hp)
        params = _flat(obj.model.state_dict())
        res = _heston_run(obj, M, N)
        _save_case(name, "heston", mode, act, [3] + layers[1:], Xi, M, N, seed, params, res,
                   Xi_full=np.array([[1.0, hp["v0"]]], np.float32), payoff=payoff, **hp)
    # train(): N schedule (Mm = 5 -> N = 5), clip 1.0, Adam, NaN skip
    torch.manual_seed(450)
    np.random.seed(450)
    with contextlib.redirect_stdout(io.StringIO()):
        obj = H(np.array([[1.0]]), 1.0, 8, 5, 1, 5.0, layers, "Naisnet", "Sine", **hp)
    p0 = _flat(obj.model.state_dict())
    np.random.seed(451)
    with contextlib.redirect_stdout(io.StringIO()):
        graph = obj.train(10, 1e-3)
    p1 = _flat(obj.model.state_dict())
    np.savez_compressed(os.path.join(OUT, "g1_train_heston_Naisnet_Sine.npz"), name="train_heston_Naisnet_Sine",
                        problem="heston", mode="Naisnet", activation="Sine", layers=np.array([3] + layers[1:]),
                        Xi=np.array([[1.0]], np.float32), Xi_full=np.array([[1.0, hp["v0"]]], np.float32), M=8,
                        N=5, T=1.0, Mm=5.0, iters=10, lr=1e-3, batch_seed=451, clip=True, params0=p0, params1=p1,
                        graph=np.asarray(graph), payoff="discontinuous", **hp)
    print(f"{'train_heston_Naisnet_Sine':42s} |dp|={np.abs(p1 - p0).max():.3e}", flush=True)


def train_cases(mods):
    """Reference train() trajectories: DeepBSDE (no clip) and nd (clip 1.0, Mm)."""
    import torch
    D = 4
    layers = [D + 1, 16, 16, 16, 16, 1]
    specs = [("train_deep_bsb_NAIS-Net_Sine", "deep", "BlackScholesBarenblatt", "bsb", "NAIS-Net", "Sine",
              np.array([1.0, 0.5] * 2)[None, :], 8, 5, None, 10, 1e-3),
             ("train_nd_call_Naisnet_Sine", "nd", "CallOption", "call", "Naisnet", "Sine",
              np.ones((1, D)), 8, 5, 5.0, 10, 1e-3)]
    for k, (name, modkey, cls, prob, mode, act, Xi, M, N, Mm, iters, lr) in enumerate(specs):
        torch.manual_seed(100 + k)
        np.random.seed(100 + k)
        C = getattr(mods[modkey], cls)
        with contextlib.redirect_stdout(io.StringIO()):
            if modkey == "deep":
                obj = C(Xi, 1.0, M, N, D, layers, mode, act)
            else:
                obj = C(Xi, 1.0, M, N, D, Mm, layers, mode, act)
        p0 = _flat(obj.model.state_dict())
        np.random.seed(200 + k)
        with contextlib.redirect_stdout(io.StringIO()):
            obj.train(iters, lr)
        p1 = _flat(obj.model.state_dict())
        np.savez_compressed(os.path.join(OUT, f"g1_{name}.npz"), name=name, problem=prob, mode=mode,
                            activation=act, layers=np.array(layers), Xi=Xi.astype(np.float32), M=M, N=N,
                            T=1.0, Mm=-1.0 if Mm is None else Mm, iters=iters, lr=lr, batch_seed=200 + k,
                            clip=modkey != "deep", params0=p0, params1=p1)
        print(f"{name:42s} |dp|={np.abs(p1 - p0).max():.3e}")


def north_star(mods, seed=0, steps=(1, 3)):
    """G2: D=100, layers [101,110x4,1] NAIS-Net Sine BSB, M=1024, N=50."""
    import torch
    D, M, N = 100, 1024, 50
    layers = [D + 1] + 4 * [110] + [1]
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    torch.manual_seed(seed)
    np.random.seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        obj = mods["deep"].BlackScholesBarenblatt(Xi, 1.0, M, N, D, layers, "NAIS-Net", "Sine")
    p0 = _flat(obj.model.state_dict())
    np.random.seed(1000 + seed)          # batch recipe: legacy MT19937 stream, seed 1000+seed
    res = _run_case(obj, M, N, D, full_z=False)
    out = dict(name="north_star", problem="bsb", mode="NAIS-Net", activation="Sine",
               layers=np.array(layers), Xi=Xi.astype(np.float32), M=M, N=N, T=1.0, seed=seed,
               batch_seed=1000 + seed, params=p0, loss=res["loss"], Y=res["Y"], grad=res["grad"],
               used=res["used"], X_sum=np.float64(res["X"].astype(np.float64).sum()),
               X_sumsq=np.float64((res["X"].astype(np.float64) ** 2).sum()), X_first=res["X"][:2])
    # reference train(): Adam, lr 1e-3, no clip, starting again from the same batch seed
    np.random.seed(1000 + seed)
    done = 0
    for s in steps:
        with contextlib.redirect_stdout(io.StringIO()):
            obj.train(s - done, 1e-3)
        done = s
        out[f"params_after_{s}"] = _flat(obj.model.state_dict())
    np.savez_compressed(os.path.join(OUT, "g2_north_star.npz"), **out)
    print(f"north_star loss={res['loss']:.6e} Y0={res['Y'][0, 0, 0]:.6f}")


def north_star_trajectory(mods, seed=0, steps=(1, 10, 100)):
    """G2b (SURVEY 8(d) accuracy): the reference DeepBSDE train() from the G2
    init and batch stream; Y0 = net_u(0, Xi) after 1/10/100 Adam steps, plus
    the parameters after 10 and 100 steps."""
    import torch
    D, M, N = 100, 1024, 50
    layers = [D + 1] + 4 * [110] + [1]
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    torch.manual_seed(seed)
    np.random.seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        obj = mods["deep"].BlackScholesBarenblatt(Xi, 1.0, M, N, D, layers, "NAIS-Net", "Sine")
    np.random.seed(1000 + seed)
    out = dict(name="north_star_trajectory", seed=seed, batch_seed=1000 + seed, steps=np.array(steps))
    y0 = []
    done = 0
    for s in steps:
        with contextlib.redirect_stdout(io.StringIO()):
            obj.train(s - done, 1e-3)
        done = s
        with torch.no_grad():
            t0 = torch.zeros(1, 1)
            x0 = torch.from_numpy(Xi).float()
            u0 = obj.model(torch.cat([t0, x0], 1))
        y0.append(float(u0))
        if s >= 10:
            out[f"params_after_{s}"] = _flat(obj.model.state_dict())
        print(f"trajectory step {s}: Y0={y0[-1]:.6f}", flush=True)
    out["Y0"] = np.array(y0)
    np.savez_compressed(os.path.join(OUT, "g2_north_star_trajectory.npz"), **out)


def round3_cases(mods):
    """Round 3: (a) the hv = false split-bf16 kernels at the north-star width --
    FC-Sine and Resnet-Sine [101,110x4,1] on DeepBSDE's BSB (DeepBSDE.py:166-178);
    (b) the with_corr / hjb train() surface: 15 iterations from iteration 490,
    crossing the it % 500 log (with_corr...py:355-453, hjb_implement.py:394-450;
    the reference HJB passes Mm=None, which cannot train, so Mm is set to N);
    (c) optimizer_type='LBFGS' through the nd train() (nd_BSPDE_case.py:347-348,
    357-361, 380-381): the closure re-evaluates on the same batch, no clip."""
    import torch
    D = 100
    L110 = [D + 1] + 4 * [110] + [1]
    xi_bsb = np.array([1.0, 0.5] * (D // 2))[None, :]
    for k, mode in enumerate(["FC", "Resnet"]):
        seed = 500 + k
        torch.manual_seed(seed)
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            obj = mods["deep"].BlackScholesBarenblatt(xi_bsb, 1.0, 16, 5, D, L110, mode, "Sine")
        params = _flat(obj.model.state_dict())
        res = _run_case(obj, 16, 5, D)
        _save_case(f"w110_deep_bsb_{mode}_Sine", "bsb", mode, "Sine", L110, xi_bsb, 16, 5, seed, params, res)

    D4 = 4
    L4 = [D4 + 1, 16, 16, 16, 16, 1]
    specs = [("train_it500_corr_basket_Naisnet_Sine", "corr", "CallOption", "basket", "Naisnet", "Sine",
              np.ones((1, D4)), {"Mm": 5.0, "correlation_type": "random_correlation"}),
             ("train_it500_hjb_Naisnet_Tanh", "hjb", "HamiltonJacobiBellman", "hjb", "Naisnet", "Tanh",
              np.zeros((1, D4)), {})]
    for k, (name, modkey, cls, prob, mode, act, Xi, kw) in enumerate(specs):
        seed = 510 + k
        torch.manual_seed(seed)
        np.random.seed(seed)
        C = getattr(mods[modkey], cls)
        with contextlib.redirect_stdout(io.StringIO()):
            if modkey == "corr":
                obj = C(Xi, 1.0, 8, 5, D4, kw["Mm"], L4, mode, act, kw["correlation_type"])
            else:
                obj = C(Xi, 1.0, 8, 5, D4, L4, mode, act)
                obj.Mm = 5.0                 # N = ceil(Mm) = 5 for it < 4000
        corr = np.asarray(obj.correlation_matrix, np.float64)
        obj.iteration = [490]
        obj.training_loss = [1.25]
        p0 = _flat(obj.model.state_dict())
        np.random.seed(520 + k)
        with contextlib.redirect_stdout(io.StringIO()):
            graph, min_loss, state, time_logs = obj.train(15, 1e-3)
        p1 = _flat(obj.model.state_dict())
        np.savez_compressed(os.path.join(OUT, f"g1_{name}.npz"), name=name, problem=prob, mode=mode,
                            activation=act, layers=np.array(L4), Xi=Xi.astype(np.float32), M=8, N=5, T=1.0,
                            Mm=5.0, iters=15, lr=1e-3, batch_seed=520 + k, start_iteration=490, start_loss=1.25,
                            params0=p0, params1=p1, graph=np.asarray(graph, np.float64), min_loss=np.float64(min_loss),
                            min_X=state[0].numpy(), min_Y=state[1].numpy(), n_time_logs=len(time_logs),
                            N_final=obj.N, corr=corr)
        print(f"{name:42s} graph={np.asarray(graph).tolist()} min_loss={min_loss:.6e}", flush=True)

    # LBFGS through the nd train(): 3 outer iterations (each up to 20 inner)
    torch.manual_seed(530)
    np.random.seed(530)
    with contextlib.redirect_stdout(io.StringIO()):
        obj = mods["nd"].CallOption(np.ones((1, D4)), 1.0, 8, 5, D4, 5.0, L4, "Naisnet", "Sine")
    p0 = _flat(obj.model.state_dict())
    np.random.seed(531)
    with contextlib.redirect_stdout(io.StringIO()):
        graph, min_loss, _ = obj.train(3, 0.05, optimizer_type="LBFGS")
    p1 = _flat(obj.model.state_dict())
    st = obj.optimizer.state[obj.optimizer._params[0]]
    np.savez_compressed(os.path.join(OUT, "g1_train_lbfgs_nd_call_Naisnet_Sine.npz"),
                        name="train_lbfgs_nd_call_Naisnet_Sine", problem="call", mode="Naisnet", activation="Sine",
                        layers=np.array(L4), Xi=np.ones((1, D4), np.float32), M=8, N=5, T=1.0, Mm=5.0, iters=3,
                        lr=0.05, batch_seed=531, params0=p0, params1=p1, min_loss=np.float64(min_loss),
                        func_evals=int(st["func_evals"]), n_iter=int(st["n_iter"]))
    print(f"{'train_lbfgs_nd_call_Naisnet_Sine':42s} |dp|={np.abs(p1 - p0).max():.3e} evals={st['func_evals']}",
          flush=True)


def round4_cases(mods):
    """Round 4: BASELINE config 1 -- the 1-D call of 1d_BSPDE_case.py
    (CallOption, 1d_BSPDE_case.py:510-560) with FC-Sine [2,256x4,1], the
    network of its __main__ (:993-1006), at M > 1 so that the D == 1 squeeze
    broadcast (Q3, :271-273) is active: a small case (M = 16, N = 5) and the
    config's full shape (M = 256, N = 50)."""
    import torch
    layers = [2] + 4 * [256] + [1]
    for k, (M, N, full_z) in enumerate([(16, 5, True), (256, 50, False)]):
        seed = 600 + k
        torch.manual_seed(seed)
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            obj = mods["oned"].CallOption(np.array([[1.0]]), 1.0, M, N, 1, 5.0, layers, "FC", "Sine")
        params = _flat(obj.model.state_dict())
        res = _run_case(obj, M, N, 1, full_z=full_z)
        _save_case(f"w256_oned_call_FC_Sine_M{M}_N{N}", "call1d", "FC", "Sine", layers, np.array([[1.0]]), M, N,
                   seed, params, res)


if __name__ == "__main__":
    m = _setup()
    if "--round4-only" in sys.argv:
        round4_cases(m)
        sys.exit(0)
    if "--round3-only" in sys.argv:
        round3_cases(m)
        sys.exit(0)
    if "--trajectory-only" in sys.argv:
        north_star_trajectory(m)
        sys.exit(0)
    if "--round2-only" in sys.argv:
        wide_cases(m)
        heston_cases(m)
        sys.exit(0)
    small_cases(m)
    round4_cases(m)
    train_cases(m)
    wide_cases(m)
    heston_cases(m)
    if "--skip-north-star" not in sys.argv:
        north_star(m)
        north_star_trajectory(m)
