"""Long-run accuracy of the plugin path (generic.py): a BlackScholesBarenblatt
subclass with sigma = 0.3 diag(X) -- an override the native coefficient table
does not take, so the subclass's own methods run -- trained with device steps
(Adam, lr 1e-3, M = 1024, N = 50, NAIS-Net 4x110 Sine).  Its exact solution
(DeepBSDE.py:345-349 with sigma = 0.3) is u(0, X0) = exp((r + sigma^2) T)
sum X0^2 = exp(0.14) 62.5 = 71.889; the parent's (sigma = 0.4) is 77.105, so
the run shows which problem was trained.

    python tools/plugin_long_run.py [--iters 20000] [--out gpurun_out/plugin_long_run.json]
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time
import warnings

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "deep-neural-network-solutions-for-partial-differential-equations_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--out", default="gpurun_out/plugin_long_run.json")
    args = ap.parse_args()
    pkg = importlib.import_module(PKG)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    class Sigma03(pkg.BlackScholesBarenblatt):
        def sigma_tf(self, t, X, Y):
            return 0.3 * torch.diag_embed(X)

    Xi = np.array([1.0, 0.5] * 50)[None, :]
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = Sigma03(Xi, 1.0, 1024, 50, 100, [101] + 4 * [110] + [1], "NAIS-Net", "Sine", device=dev)
    assert not m.native_coefficients
    exact03 = math.exp(0.05 + 0.3 ** 2) * float(np.sum(Xi ** 2))
    exact04 = math.exp(0.05 + 0.4 ** 2) * float(np.sum(Xi ** 2))
    opt = m.new_optimizer_state("Adam", 1e-3)
    trace = []
    start = time.perf_counter()
    for it in range(args.iters):
        loss = m.device_step(opt, 1e-3, seed=it)
        if (it + 1) % 1000 == 0 or it == 0:
            with torch.no_grad():
                u0 = float(m.net_u(torch.zeros(1), m.Xi.reshape(1, -1))[0])
            trace.append({"iter": it + 1, "loss": float(loss), "u0": u0})
            print(json.dumps(trace[-1]), flush=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - start
    u0 = trace[-1]["u0"]
    res = {"problem": "BlackScholesBarenblatt subclass, sigma = 0.3 diag(X) (generic path)",
           "generic_reason": m.generic_reason, "iters": args.iters, "M": 1024, "N": 50,
           "u0": u0, "u0_exact_sigma03": exact03, "abs_err": abs(u0 - exact03), "rel_err": abs(u0 - exact03) / exact03,
           "u0_exact_parent_sigma04": exact04, "s_per_iter": el / args.iters, "trace": trace}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "trace"}))


if __name__ == "__main__":
    main()
