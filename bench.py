"""Benchmark: deep-BSDE training step, 100-D Black-Scholes-Barenblatt
(BASELINE.json configs[1]: NAIS-Net [101,110,110,110,110,1], Sine, batch 1024
paths per GPU, N = 50 time steps, T = 1, Adam lr 1e-3, DeepBSDE.py semantics).

One step = one optimizer iteration over one synthetic minibatch: Brownian
increments drawn on the device (Philox), Euler-Maruyama rollout, network
forward + Z, residual loss, second-order backward, [RCCL all-reduce], Adam.
All inputs resident in HBM.  value = total SDE path-steps/s over all ranks
(weak scaling: 1024 paths per GPU; --strong: 1024 paths in total, split).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--workload oned|basket|hjb|heston runs BASELINE configs 1 and 3-5 on this
process's GPUs (separate lines for DESIGN.md; the headline is the default bsb
workload).
"""
from __future__ import annotations

import argparse
import csv
import glob
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "deep-neural-network-solutions-for-partial-differential-equations_amd"

D, W_HID, N_STEPS, M_PER_GPU, T = 100, 110, 50, 1024, 1.0
LAYERS = [D + 1] + 4 * [W_HID] + [1]
LR = 1e-3
U0_EXACT = float(np.exp((0.05 + 0.4 ** 2) * 1.0) * 62.5)     # DeepBSDE.py:345-349 at Xi=[1,.5]*50
PEAK_FP32_MFMA_TFLOPS = 157.3                                # MI355X_MICROARCH.md, dense f32 MFMA
# split-bf16 kernels (solver.matrix_form): an fp32 product block costs six dense
# bf16 MFMAs, so their fp32-equivalent matrix peak is the dense bf16 peak / 6
PEAK_BF16_DENSE_TFLOPS = 2500.0
PEAK_X3_TFLOPS = PEAK_BF16_DENSE_TFLOPS / 6.0
X3_RECORDS = {1: ("fused_phases_pipelined", "fused_fwd_inputgrad", "fused_tangent_reverse"), 2: ("tn_weight_grad",),
              4: ("gemm_",)}
PEAK_HBM_GBS = 8000.0
PROFILE_ROUND = "r6"          # profiles/<round>_pmc_* counter collections of the current build
# rocprof symbol of each profiled launch class (EPI ids from csrc/kernels.hpp)
KERNEL_SYMBOL = {
    "gemm_xstack_fwd": "chain_gemm_kernel<7, 0>", "gemm_block_fwd": "chain_gemm_kernel<7, 1>",
    "gemm_block_inputgrad": "chain_gemm_kernel<7, 2>", "gemm_z_cotangent": "chain_gemm_kernel<7, 3>",
    "gemm_xstack_tangent": "chain_gemm_kernel<7, 4>", "gemm_block_tangent": "chain_gemm_kernel<7, 5>",
    "gemm_block_reverse": "chain_gemm_kernel<7, 6>", "tn_weight_grad": "tnw_kernel",
    "fused_fwd_inputgrad": "phaseA_kernel", "fused_tangent_reverse": "phaseC_kernel",
    "fused_phases_pipelined": ("phaseA_kernel", "phaseC_kernel"),
    "rollout": "rollout_kernel", "grad_finalize": "tilefin_kernel",
}
KERNEL_SYMBOL_X3 = {"tn_weight_grad": "tnw_x3_kernel"}   # when matrix_form bit 1 is set
# the profile records that time MFMA work.  fused_phases_pipelined is one
# record per step for both phase kernels: two path chunks on two streams,
# events around the whole section (its kernels overlap, so per-launch times
# of a single kernel would not add up to the step)
MFMA_LAUNCHES = ("fused_phases_pipelined", "fused_fwd_inputgrad", "fused_tangent_reverse", "tn_weight_grad", "gemm_")

# BASELINE.json configs (the headline is "bsb")
WORKLOADS = {
    "bsb": dict(cls="BlackScholesBarenblatt", D=100, layers=[101] + 4 * [110] + [1], mode="NAIS-Net",
                act="Sine", M=1024, N=50, xi="bsb",
                desc="100-D Black-Scholes-Barenblatt deep-BSDE training step (DeepBSDE.py semantics: Adam lr "
                     "1e-3, no clip)"),
    "basket": dict(cls="BasketCallOption", D=100, layers=[101] + 4 * [110] + [1], mode="Naisnet", act="ReLU",
                   M=4096, N=50, xi="ones",
                   desc="100-D basket call, Cholesky-correlated device increments (Q10 matrix), Naisnet-ReLU "
                        "(with_corr_high_dimension_pde.py semantics: Adam, clip 1.0)"),
    "hjb": dict(cls="HamiltonJacobiBellman", D=100, layers=[101] + 4 * [256] + [1], mode="FC", act="Sine",
                M=2048, N=20, xi="zeros", desc="100-D HJB, FC-Sine [101,256x4,1] (hjb_implement.py semantics)"),
    "oned": dict(cls="CallOption1D", D=1, layers=[2] + 4 * [256] + [1], mode="FC", act="Sine", M=256, N=50,
                 xi="ones", desc="1-D Black-Scholes call, FC-Sine [2,256x4,1], batch 256, 50 steps, Q3 squeeze "
                                 "broadcast active (1d_BSPDE_case.py semantics: Adam, clip 1.0)"),
    "heston": dict(cls="HestonFBSNN", D=50, layers=[51] + 4 * [110] + [1], mode="Naisnet", act="Sine",
                   M=1024, N=100, xi="ones",
                   desc="50-asset Heston (state 100), Naisnet-Sine (heston_dnnpde.py semantics generalised to "
                        "k assets: clamps, u >= 0, NaN skip, clip 1.0)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(iters=30, warmup=2):
    """The oracle's faithful torch-CPU restatement of the reference step
    (fetch_minibatch + loss_function + double backward + Adam, anomaly mode
    off), timed on the host cores: `warmup` untimed iterations, then `iters`
    timed ones; median and spread reported."""
    from oracle import fbsnn_ref as fr
    torch.manual_seed(0)
    np.random.seed(0)
    model = fr.build_model("NAIS-Net", LAYERS, "Sine")
    prob = fr.make_problem("bsb", D)
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    times = []
    for i in range(warmup + iters):
        t0 = time.time()
        fr.train(model, prob, Xi, M_PER_GPU, N_STEPS, D, T, 1, LR, clip=False)
        if i >= warmup:
            times.append(time.time() - t0)
    med = float(np.median(times))
    return {"value": M_PER_GPU * N_STEPS / med, "unit": "path-steps/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{iters} timed training iterations after {warmup} warm-up of the same workload (M=1024, "
                      f"N=50, D=100, NAIS-Net 4x110 Sine, Adam) by oracle/fbsnn_ref.py (torch CPU, autograd "
                      f"double backward, dense diag sigma, anomaly off): median {med:.3f} s/iteration, "
                      f"min {min(times):.3f}, max {max(times):.3f}",
            "s_per_iter": {"median": med, "min": float(min(times)), "max": float(max(times)),
                           "p25": float(np.percentile(times, 25)), "p75": float(np.percentile(times, 75)),
                           "n": len(times)}}


def parity_trajectory(pkg, dev):
    """The north-star accuracy metric: Y0 = u(0, X0) after 1, 10
    and 100 steps of the native train() -- the reference's DeepBSDE train()
    semantics (fresh Adam per call, lr 1e-3, no clip) from the reference's own
    init and numpy batch stream -- against the reference's Y0 on the same
    steps (tests/golden/g2_north_star_trajectory.npz, produced by the
    reference itself).  The train() progress prints go to stderr."""
    import contextlib
    golden = os.path.join(ROOT, "tests", "golden")
    g = np.load(os.path.join(golden, "g2_north_star.npz"))
    tr = np.load(os.path.join(golden, "g2_north_star_trajectory.npz"))
    layers = [int(v) for v in g["layers"]]
    Dg, Mg, Ng = layers[0] - 1, int(g["M"]), int(g["N"])
    m = pkg.BlackScholesBarenblatt(g["Xi"], float(g["T"]), Mg, Ng, Dg, layers, "NAIS-Net", "Sine", device=dev)
    m.params.copy_(torch.from_numpy(g["params"]).to(dev))
    np.random.seed(int(tr["batch_seed"]))
    t0 = torch.zeros(1, device=dev)
    x0 = torch.from_numpy(g["Xi"]).to(dev).reshape(1, Dg)
    rows, done = [], 0
    with contextlib.redirect_stdout(sys.stderr):
        for s, y_ref in zip(tr["steps"], tr["Y0"]):
            m.train(int(s) - done, 1e-3)
            done = int(s)
            with torch.no_grad():
                u = float(m.net_u(t0, x0)[0])
            rows.append({"steps": int(s), "Y0": u, "Y0_reference": float(y_ref), "abs_err": abs(u - float(y_ref))})
    return {"metric": "|u(0,X_0) - reference| after k reference train() steps (same init, same numpy batches)",
            "tolerance": 1e-3, "max_abs_err": max(r["abs_err"] for r in rows), "points": rows}


def traffic_from_pmc(symbol, launches_per_step):
    """HBM bytes per launch of `symbol` (or per record of a tuple of symbols:
    the sum over them, each at its launches per record) from a committed
    rocprofv3 --pmc counter collection (profiles/<round>_pmc*counter_collection.csv):
    FETCH_SIZE is doubled (gfx950 reports half of wide coalesced reads,
    MI355X_MICROARCH.md HBM section), WRITE_SIZE taken as is; both in KB.
    The counter runs use the same bench command, so a kernel's launches per
    step there equal the timed run's."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"{PROFILE_ROUND}_pmc*counter_collection.csv")))
    if not files:
        return None
    symbols = symbol if isinstance(symbol, tuple) else (symbol,)
    total = 0.0
    for sym in symbols:
        sums = {"FETCH_SIZE": [], "WRITE_SIZE": []}
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if sym in row.get("Kernel_Name", "") and row.get("Counter_Name") in sums:
                        sums[row["Counter_Name"]].append(float(row["Counter_Value"]))
        if not sums["FETCH_SIZE"] or not sums["WRITE_SIZE"]:
            return None
        per_launch = 1024.0 * (2.0 * np.mean(sums["FETCH_SIZE"]) + np.mean(sums["WRITE_SIZE"]))
        # launches of this symbol per record: the phase kernels run once per chunk
        n = 2.0 if len(symbols) > 1 else 1.0
        total += per_launch * n
    return total


def build_model(pkg, wl, M, dev, args):
    cls = getattr(pkg, wl["cls"])
    Dw = wl["D"]
    if wl["xi"] == "bsb":
        Xi = np.array([1.0, 0.5] * (Dw // 2))[None, :]
    elif wl["xi"] == "zeros":
        Xi = np.zeros((1, Dw))
    else:
        Xi = np.ones((1, Dw))
    mode = args.mode or wl["mode"]
    act = args.activation or wl["act"]
    if wl["cls"] == "BlackScholesBarenblatt":
        return cls(Xi, T, M, wl["N"], Dw, wl["layers"], mode, act, device=dev), Xi
    if wl["cls"] == "HamiltonJacobiBellman":
        return cls(Xi, T, M, wl["N"], Dw, wl["layers"], mode, act, device=dev), Xi
    if wl["cls"] == "CallOption1D":
        m = cls(Xi, T, M, wl["N"], Dw, None, wl["layers"], mode, act, device=dev)
        m.N = wl["N"]
        return m, Xi
    if wl["cls"] == "BasketCallOption":
        np.random.seed(0)                      # the Q10 correlation matrix draw
        m = cls(Xi, T, M, wl["N"], Dw, None, wl["layers"], mode, act, "random_correlation", device=dev)
        m.N = wl["N"]
        return m, Xi
    return cls(Xi, T, M, wl["N"], Dw, None, wl["layers"], mode, act, device=dev), Xi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)      # >= 50 steps after >= 10 warm-up
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--strong", action="store_true", help="global batch fixed at the workload's M (split)")
    ap.add_argument("--workload", default="bsb", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-iters", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the 100-step Y0 parity trajectory")
    ap.add_argument("--paths-per-gpu", type=int, default=None,
                    help="paths per GPU (default: the workload's M); e.g. 128/256/512 = the per-rank shapes of "
                         "8/4/2-GPU strong scaling")
    ap.add_argument("--no-prefetch", action="store_true", help="A/B: roll each step's paths out in the step itself")
    ap.add_argument("--activation", default=None, help="experiments only; the headline is Sine")
    ap.add_argument("--mode", default=None, help="experiments only; the headline is NAIS-Net")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    wl = WORKLOADS[args.workload]
    pkg = importlib.import_module(PKG)
    torch.manual_seed(0)
    M_work = args.paths_per_gpu or wl["M"]
    M_global = M_work if args.strong else M_work * world
    model, Xi = build_model(pkg, wl, M_global, dev, args)
    opt = model.new_optimizer_state("Adam", LR)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    it = 0
    # each step prefetches the next step's device rollout (device_step next_seed)
    for _ in range(args.warmup):
        model.device_step(opt, LR, seed=it, next_seed=None if args.no_prefetch else it + 1)
        it += 1
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = model.device_step(opt, LR, seed=it, next_seed=None if args.no_prefetch else it + 1)
        it += 1
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e)
    final_loss = float(loss)

    # the one collective per step, alone: [grad | loss] all-reduce latency
    allreduce_us = None
    if world > 1:
        buf = model._gradbuf.clone()
        for _ in range(5):
            dist.all_reduce(buf)
        barrier()
        ta = time.perf_counter()
        for _ in range(20):
            dist.all_reduce(buf)
        barrier()
        allreduce_us = 1e6 * (time.perf_counter() - ta) / 20

    # per-kernel HIP-event timing of the same K steps (separate window so the
    # headline time carries no event overhead)
    model.solver.profile(True)
    model.solver.profile_reset()
    for _ in range(args.steps):
        model.device_step(opt, LR, seed=it, next_seed=None if args.no_prefetch else it + 1)
        it += 1
    prof = model.solver.profile_read()
    model.solver.profile(False)

    with torch.no_grad():
        u0, _ = model.net_u(torch.zeros(1), model.Xi.reshape(1, -1))
    u0 = float(u0)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    ms_per_step = 1000.0 * elapsed / args.steps
    total_path_steps = M_global * wl["N"]
    value = total_path_steps * args.steps / elapsed

    # roofline of the dominant MFMA kernel (the main-stream network passes;
    # side-stream launches such as loss_final include queue wait in their events)
    mfma = {k: v for k, v in prof.items() if k.startswith(MFMA_LAUNCHES)}
    name, st = max(mfma.items(), key=lambda kv: kv[1]["ms"])
    form = model.solver.matrix_form

    def peak_of(rec):
        """(peak, form text) of a record's matrix instruction: the split-bf16
        kernels against the bf16 dense peak / 6 (fp32-equivalent FLOPs), the
        fp32-input MFMA kernels against the fp32 MFMA peak"""
        for bit, recs in X3_RECORDS.items():
            if form & bit and rec.startswith(recs):
                return PEAK_X3_TFLOPS, "split-bf16 (6 x v_mfma_f32_16x16x32_bf16 per fp32 block, fp32-accurate)"
        return PEAK_FP32_MFMA_TFLOPS, "fp32-input MFMA (v_mfma_f32_16x16x4_f32)"

    def sym_of(rec):
        if form & 2 and rec in KERNEL_SYMBOL_X3:
            # the chain layouts' split-bf16 weight-gradient tiles (tnx3.hpp)
            return "tn_x3_kernel" if (form & 4 and rec == "tn_weight_grad") else KERNEL_SYMBOL_X3[rec]
        return KERNEL_SYMBOL.get(rec, rec)

    avg_ms = st["ms"] / st["launches"]
    achieved = st["flops"] / st["launches"] / (avg_ms * 1e-3) / 1e12
    symbol = sym_of(name)
    traffic = traffic_from_pmc(symbol, st["launches"] / args.steps) if args.workload == "bsb" else None
    symtxt = " + ".join(symbol) if isinstance(symbol, tuple) else symbol
    peak, form_txt = peak_of(name)
    roofline = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                "frac": achieved / peak, "traffic": traffic, "kernel": f"{name} ({symtxt})",
                "matrix_form": form_txt, "frac_of_fp32_mfma_peak": achieved / PEAK_FP32_MFMA_TFLOPS,
                "avg_launch_ms": avg_ms, "launches_per_step": st["launches"] / args.steps,
                "alg_flops_per_launch": st["flops"] / st["launches"]}
    # every other MFMA record, same definition (e.g. the weight-gradient kernel)
    roofline_others = {}
    for k, v in mfma.items():
        if k == name:
            continue
        a_ms = v["ms"] / v["launches"]
        a_tf = v["flops"] / v["launches"] / (a_ms * 1e-3) / 1e12
        pk, ftxt = peak_of(k)
        roofline_others[k] = {"achieved": a_tf, "peak": pk, "frac": a_tf / pk, "matrix_form": ftxt,
                              "avg_launch_ms": a_ms,
                              "traffic": traffic_from_pmc(sym_of(k), 1.0)
                              if args.workload == "bsb" else None}
    # the path-step kernel against HBM (north_star: achieved GB/s of the path step)
    rp = prof.get("rollout")
    roofline_path = None
    if rp:
        r_ms = rp["ms"] / rp["launches"]
        gbs = rp["bytes"] / rp["launches"] / (r_ms * 1e-3) / 1e9
        roofline_path = {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": gbs / PEAK_HBM_GBS, "kernel": "rollout", "avg_launch_ms": r_ms,
                         "alg_bytes_per_launch": rp["bytes"] / rp["launches"],
                         "traffic": traffic_from_pmc("rollout", 1.0) if args.workload == "bsb" else None}
    step_flops = sum(v["flops"] for v in prof.values()) / args.steps
    breakdown = {k: round(v["ms"] / args.steps, 4) for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])}

    cpu = None
    if world == 1 and not args.no_cpu_baseline and args.workload == "bsb":
        cpu = cpu_baseline(args.cpu_iters)
    parity = None
    if not args.no_parity and args.workload == "bsb":
        parity = parity_trajectory(pkg, dev)

    Mloc = M_global // world
    out = {
        "metric": "SDE-path-steps/sec + |u(0,X_0) err|, 100-D BSB, 1/2/4/8 MI355X",
        "value": value,
        "unit": "path-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: device Philox Brownian increments, reference (xavier) init weights, seed 0",
        "config": {"workload": wl["desc"], "name": args.workload, "D": wl["D"], "layers": wl["layers"],
                   "mode": args.mode or wl["mode"], "activation": args.activation or wl["act"],
                   "paths_per_gpu": Mloc, "global_batch": M_global, "time_steps": wl["N"],
                   "parallelism": f"dp{world}"},
        "roofline": roofline,
        "roofline_other_mfma": roofline_others,
        "roofline_path_step": roofline_path,
        "allreduce_us": allreduce_us,
        "per_gpu_path_steps_per_s": value / world,
        "step_alg_tflops": step_flops / (ms_per_step * 1e-3) / 1e12,
        "step_kernel_ms": breakdown,
        "accuracy": {"parity": parity,
                     "abs_err": parity["max_abs_err"] if parity else None,
                     "bench_model": {"u0": u0, "train_iterations": it, "final_loss": final_loss,
                                     "u0_exact": U0_EXACT if args.workload == "bsb" else None,
                                     "exact_gap": abs(u0 - U0_EXACT) if args.workload == "bsb" else None,
                                     "note": "u(0,X0) of the benchmark's own model after its few timed steps; the "
                                             "exact value 77.1049 (DeepBSDE.py:345-349) needs ~2e4 iterations"}},
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
