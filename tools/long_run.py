"""Long-run accuracy of the native training path against the reference's
published result and the north star's exact value (VERDICT r4
item 2).

The reference's run_model (DeepBSDE.py:352-427, invoked at :447 as
run_model(model, 2*10**4, 1e-3)) trains with DeepBSDE.FBSNN.train
(DeepBSDE.py:265-295: Adam, no clip, a fresh numpy batch per iteration),
then draws the seed-42 batch (np.random.seed(42); fetch_minibatch,
:363-365), predicts on it and plots errors = sqrt((Y_test - Y_pred)^2 /
Y_test^2) against u_exact (:345-349, :410-411), mean and mean + 2 std over
the paths at every t.  The published figure (FC-Sine [101,256x4,1], M = 100,
N = 50, D = 100) reads ~0.018 at t = 0, ~0.026 peak mean over t and ~0.034
peak mean + 2 std.

Cases (each a fresh model, torch.manual_seed(seed) init):
  fc256    the published configuration: FC-Sine [101,256x4,1], M = 100
  north    the north star: NAIS-Net-Sine [101,110x4,1], M = 1024
Both at N = 50, T = 1, Xi = [1, 0.5] x 50, lr 1e-3, 2e4 iterations.

Training increments: --stream device (default) draws them on the device
(Philox, same N(0, dt) law; the throughput path, bench.py's step) with the
update fused into the gradient finalize; --stream host runs the package's
train() -- the reference's own numpy stream and per-iteration loss sync,
iteration for iteration the reference's loop.  The evaluation batch is the
reference's seed-42 numpy batch either way.

    python tools/long_run.py [--cases fc256,north] [--iters 20000] [--seeds 0]
                             [--stream device|host] [--out profiles/r5_long_run.json]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "deep-neural-network-solutions-for-partial-differential-equations_amd"

D, N, T = 100, 50, 1.0
U0_EXACT = float(np.exp((0.05 + 0.4 ** 2) * T) * 62.5)   # u_exact(0, Xi), DeepBSDE.py:345-349
CASES = {
    "fc256": dict(layers=[D + 1] + 4 * [256] + [1], mode="FC", act="Sine", M=100),
    "north": dict(layers=[D + 1] + 4 * [110] + [1], mode="NAIS-Net", act="Sine", M=1024),
}
PUBLISHED = {"mean_t0": 0.018, "peak_mean": 0.026, "peak_mean_2std": 0.034,
             "source": "100-dimensional Black-Scholes-Barenblatt, FC-Sine.png (DeepBSDE.py:410-426), BASELINE.md"}


def evaluate(pkg, model, Xi):
    """run_model's evaluation (DeepBSDE.py:363-365, 345-349, 410-413)."""
    np.random.seed(42)
    t_test, W_test = model.fetch_minibatch()
    X_pred, Y_pred = model.predict(Xi, t_test, W_test)
    t_test = t_test.cpu().numpy()
    X_pred = X_pred.cpu().numpy()
    Y_pred = Y_pred.cpu().numpy()
    M = t_test.shape[0]
    Y_test = np.reshape(pkg.deepbsde.u_exact(np.reshape(t_test[0:M], [-1, 1]), np.reshape(X_pred[0:M], [-1, D]), T),
                        [M, -1, 1])
    errors = np.sqrt((Y_test - Y_pred) ** 2 / Y_test ** 2)
    mean_e = np.mean(errors, 0)[:, 0]
    std_e = np.std(errors, 0)[:, 0]
    return {"mean_t0": float(mean_e[0]), "mean_T": float(mean_e[-1]), "peak_mean": float(mean_e.max()),
            "peak_mean_2std": float((mean_e + 2 * std_e).max()), "mean_over_t": float(mean_e.mean()),
            "mean_by_t": [round(float(v), 6) for v in mean_e]}


def run_case(pkg, name, seed, iters, stream, dev):
    cfg = CASES[name]
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    torch.manual_seed(seed)
    np.random.seed(seed)
    model = pkg.deepbsde.BlackScholesBarenblatt(Xi, T, cfg["M"], N, D, cfg["layers"], cfg["mode"], cfg["act"],
                                                device=dev)
    model.log_print = False
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if stream == "host":
        graph = model.train(iters, 1e-3)
        losses = graph[1]
    else:
        graph = model.train_device(iters, 1e-3, seed=seed)
        losses = graph[1]
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    with torch.no_grad():
        u0, _ = model.net_u(torch.zeros(1), model.Xi.reshape(1, -1))
    u0 = float(u0)
    ev = evaluate(pkg, model, Xi)
    rec = {"case": name, "layers": cfg["layers"], "mode": cfg["mode"], "activation": cfg["act"], "M": cfg["M"],
           "N": N, "seed": seed, "iterations": iters, "lr": 1e-3, "stream": stream, "train_wall_s": round(wall, 3),
           "ms_per_iteration": round(1e3 * wall / iters, 4), "u0": u0, "u0_exact": U0_EXACT,
           "u0_abs_err": abs(u0 - U0_EXACT), "u0_rel_err": abs(u0 - U0_EXACT) / U0_EXACT,
           "final_window_loss": float(losses[-1]), "seed42_rel_error": ev}
    print(json.dumps({k: v for k, v in rec.items() if k != "seed42_rel_error"}
                     | {"seed42": {k: v for k, v in ev.items() if k != "mean_by_t"}}), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="fc256,north")
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--seeds", default="0")
    ap.add_argument("--stream", choices=("device", "host"), default="device")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    pkg = importlib.import_module(PKG)
    dev = torch.device("cuda:0")
    recs = [run_case(pkg, c, int(s), args.iters, args.stream, dev)
            for c in args.cases.split(",") for s in args.seeds.split(",")]
    summary = {"published_fc256": PUBLISHED, "u0_exact": U0_EXACT, "runs": recs}
    fc = [r for r in recs if r["case"] == "fc256"]
    if fc:
        m0 = float(np.mean([r["seed42_rel_error"]["mean_t0"] for r in fc]))
        summary["fc256_vs_published"] = {
            "mean_t0": m0, "ratio_to_published": m0 / PUBLISHED["mean_t0"],
            "peak_mean": float(np.mean([r["seed42_rel_error"]["peak_mean"] for r in fc])),
            "peak_mean_2std": float(np.mean([r["seed42_rel_error"]["peak_mean_2std"] for r in fc]))}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "runs"}))


if __name__ == "__main__":
    main()
