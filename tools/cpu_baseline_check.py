"""Container-only check of bench.py's cpu_baseline leg:
the oracle's torch-CPU restatement (oracle/fbsnn_ref.py) must reproduce the
imported reference's training iteration (DeepBSDE.py BlackScholesBarenblatt,
NAIS-Net [101,110x4,1], Sine, M=1024, N=50, Adam, anomaly mode off) in value
and within +-10 % in time on the same cores.

Reads /root/reference, so it runs in the build container only; the result is
committed as profiles/r2_cpu_baseline_check.json.

    python tools/cpu_baseline_check.py [--iters 6] [--warmup 1]
"""
from __future__ import annotations

import argparse
import contextlib
import importlib.util
import io
import json
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, ROOT)


def load_reference():
    import matplotlib
    matplotlib.use("Agg")
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
    sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location("ref_DeepBSDE", os.path.join(REF, "DeepBSDE.py"))
    mod = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()):
        spec.loader.exec_module(mod)
    torch.autograd.set_detect_anomaly(False)     # DeepBSDE.py:11 turns it on
    return mod


def time_iters(step, iters, warmup):
    ts = []
    for i in range(warmup + iters):
        t0 = time.perf_counter()
        step()
        if i >= warmup:
            ts.append(time.perf_counter() - t0)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    from oracle import fbsnn_ref as fr
    D, M, N = 100, 1024, 50
    layers = [D + 1] + 4 * [110] + [1]
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    ref = load_reference()

    # same init, same batch stream: one iteration of each must agree
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        obj = ref.BlackScholesBarenblatt(Xi, 1.0, M, N, D, layers, "NAIS-Net", "Sine")
    model = fr.build_model("NAIS-Net", layers, "Sine")
    fr.set_flat_params(model, fr.flat_params(obj.model))
    np.random.seed(7)
    with contextlib.redirect_stdout(io.StringIO()):
        obj.train(1, 1e-3)
    np.random.seed(7)
    fr.train(model, fr.make_problem("bsb", D), Xi, M, N, D, 1.0, 1, 1e-3, clip=False)
    dp = float(np.abs(fr.flat_params(model) - fr.flat_params(obj.model)).max())

    def ref_step():
        with contextlib.redirect_stdout(io.StringIO()):
            obj.train(1, 1e-3)

    def port_step():
        fr.train(model, fr.make_problem("bsb", D), Xi, M, N, D, 1.0, 1, 1e-3, clip=False)

    # interleaved, so machine drift hits both legs alike
    t_ref, t_port = [], []
    for i in range(args.warmup + args.iters):
        a = time_iters(ref_step, 1, 0)[0]
        b = time_iters(port_step, 1, 0)[0]
        if i >= args.warmup:
            t_ref.append(a)
            t_port.append(b)
    mr, mp = float(np.median(t_ref)), float(np.median(t_port))
    out = {"threads": torch.get_num_threads(), "iters": args.iters, "warmup": args.warmup,
           "reference_s_per_iter": {"median": mr, "min": min(t_ref), "max": max(t_ref)},
           "port_s_per_iter": {"median": mp, "min": min(t_port), "max": max(t_port)},
           "port_over_reference_time": mp / mr, "within_10pct": abs(mp / mr - 1) <= 0.10,
           "max_abs_param_diff_after_1_iter": dp,
           "reference_path_steps_per_s": M * N / mr, "port_path_steps_per_s": M * N / mp}
    print(json.dumps(out, indent=1))
    with open(os.path.join(ROOT, "profiles", "r2_cpu_baseline_check.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
