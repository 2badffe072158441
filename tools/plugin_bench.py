"""Step time of the plugin path (generic.py) beside the native one at the
north-star shape (100-D BSB, NAIS-Net 4x110 Sine, M = 1024, N = 50, Adam):

  native   BlackScholesBarenblatt (its problem_spec runs in the kernels)
  plugin   a BlackScholesBarenblatt subclass overriding sigma_tf with the SAME
           formula written differently (0.4 * diag_embed(X)) -- the override
           check finds no disagreement, so it stays native (control)
  generic  the subclass with sigma = 0.3 diag(X): torch rollout + residuals on
           the device, u / Z and the network backward through dbsde_net_u /
           dbsde_net_u_vjp

Each: --warmup device_step()s, then --steps timed ones (synchronised), one
JSON line per variant.

    python tools/plugin_bench.py [--steps 50] [--warmup 10]
"""
from __future__ import annotations

import argparse
import importlib
import json
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
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--paths", type=int, default=1024)
    args = ap.parse_args()
    pkg = importlib.import_module(PKG)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    class SameSigma(pkg.BlackScholesBarenblatt):
        def sigma_tf(self, t, X, Y):
            return 0.4 * torch.diag_embed(X)

    class Sigma03(pkg.BlackScholesBarenblatt):
        def sigma_tf(self, t, X, Y):
            return 0.3 * torch.diag_embed(X)

    Xi = np.array([1.0, 0.5] * 50)[None, :]
    layers = [101] + 4 * [110] + [1]
    M, N = args.paths, 50
    for name, cls in (("native", pkg.BlackScholesBarenblatt), ("plugin_same_spec", SameSigma),
                      ("generic", Sigma03)):
        torch.manual_seed(0)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            m = cls(Xi, 1.0, M, N, 100, layers, "NAIS-Net", "Sine", device=dev)
        opt = m.new_optimizer_state("Adam", 1e-3)
        it = 0
        for _ in range(args.warmup):
            m.device_step(opt, 1e-3, seed=it, next_seed=it + 1)
            it += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = m.device_step(opt, 1e-3, seed=it, next_seed=it + 1)
            it += 1
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / args.steps
        print(json.dumps({"variant": name, "native_coefficients": bool(m.native_coefficients),
                          "generic_reason": m.generic_reason, "M": M, "N": N, "ms_per_step": ms,
                          "path_steps_per_s": M * N / (ms * 1e-3), "final_loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
