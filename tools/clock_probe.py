"""Clock / power samples beside per-step times.

Runs the headline bench loop (bsb, M = 1024, N = 50, prefetched device steps)
for --steps steps after --warmup, records a HIP event on the main stream after
every step (the step's work is joined into that stream), and samples the
GPU's current SCLK / MCLK / FCLK levels and power from sysfs in a thread every
--period ms meanwhile.  Prints per-window means (steps 5-18 vs 50-78 by
default: the windows of profiles/r5_window.txt) and writes the raw series as
JSON.

    python tools/clock_probe.py [--steps 100] [--warmup 0] [--out gpurun_out/clocks.json]
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import importlib
import json
import os
import re
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "deep-neural-network-solutions-for-partial-differential-equations_amd"


def sysfs_dir(dev_index):
    """/sys/bus/pci/devices/<bdf> of the torch device (its PCI address)."""
    p = torch.cuda.get_device_properties(dev_index)
    bus, devn, dom = getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", 0), getattr(p, "pci_domain_id", 0)
    if bus is None:
        return None
    d = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{devn:02x}.0"
    return d if os.path.isdir(d) else None


def current_level(path):
    """The '*'-marked frequency of a pp_dpm_* file, in MHz."""
    try:
        with open(path) as f:
            for line in f:
                if "*" in line:
                    m = re.search(r"(\d+)\s*[Mm]hz", line)
                    return int(m.group(1)) if m else None
    except OSError:
        return None
    return None


def read_num(path, scale):
    try:
        with open(path) as f:
            return float(f.read().strip()) * scale
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--period", type=float, default=1.0, help="sampling period, ms")
    ap.add_argument("--out", default="gpurun_out/clocks.json")
    ap.add_argument("--windows", default="5-18,50-78")
    args = ap.parse_args()

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    base = sysfs_dir(0)
    hw = sorted(glob.glob(os.path.join(base, "hwmon", "hwmon*"))) if base else []
    hw = hw[0] if hw else None
    files = {}
    if base:
        for k in ("sclk", "mclk", "fclk", "socclk"):
            f = os.path.join(base, f"pp_dpm_{k}")
            if os.path.exists(f):
                files[k] = ("dpm", f)
    if hw:
        for k, name, sc in (("sclk_in", "freq1_input", 1e-6), ("mclk_in", "freq2_input", 1e-6),
                            ("power_avg_w", "power1_average", 1e-6), ("power_in_w", "power1_input", 1e-6),
                            ("temp_edge_c", "temp1_input", 1e-3), ("temp_hot_c", "temp2_input", 1e-3),
                            ("temp_mem_c", "temp3_input", 1e-3)):
            f = os.path.join(hw, name)
            if os.path.exists(f):
                files[k] = ("num", f, sc)
    print("sysfs:", base, hw, sorted(files), file=sys.stderr)

    pkg = importlib.import_module(PKG)
    torch.manual_seed(0)
    Xi = np.array([1.0, 0.5] * 50)[None, :]
    m = pkg.BlackScholesBarenblatt(Xi, 1.0, 1024, 50, 100, [101] + 4 * [110] + [1], "NAIS-Net", "Sine", device=dev)
    opt = m.new_optimizer_state("Adam", 1e-3)

    samples, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            t = time.perf_counter()
            row = {"t": t}
            for k, spec in files.items():
                row[k] = current_level(spec[1]) if spec[0] == "dpm" else read_num(spec[1], spec[2])
            samples.append(row)
            time.sleep(args.period * 1e-3)

    # in-kernel clock between steps (tools/ubench/clockstamp.hip; build:
    # hipcc -O3 --offload-arch=gfx950 -fPIC -shared -o tools/ubench/libclockstamp.so tools/ubench/clockstamp.hip)
    cs_path = os.path.join(ROOT, "tools", "ubench", "libclockstamp.so")
    cs = ctypes.CDLL(cs_path) if os.path.exists(cs_path) else None
    stamps = torch.zeros(2 * (args.steps + 1), dtype=torch.int64, device=dev)
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    time.sleep(0.05)
    it = 0
    for _ in range(args.warmup):
        m.device_step(opt, 1e-3, seed=it, next_seed=it + 1)
        it += 1
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    host0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        m.device_step(opt, 1e-3, seed=it, next_seed=it + 1)
        evs[k].record(stream)
        if cs is not None:
            cs.clockstamp_launch(ctypes.c_void_p(stamps.data_ptr()), k, ctypes.c_void_p(stream.cuda_stream))
        it += 1
    torch.cuda.synchronize()
    time.sleep(0.02)
    stop.set()
    th.join()
    ends = np.array([ev0.elapsed_time(e) for e in evs])          # ms since ev0
    dur = np.diff(np.concatenate([[0.0], ends]))
    # host time of each step's end (ev0 recorded right after a synchronize)
    t_end = host0 + ends * 1e-3
    t_start = np.concatenate([[host0], t_end[:-1]])
    keys = sorted(files)
    st = stamps.cpu().numpy().reshape(-1, 2)
    rows = []
    for k in range(args.steps):
        ss = [s for s in samples if t_start[k] <= s["t"] < t_end[k]]
        if not ss:   # nearest sample
            ss = [min(samples, key=lambda s: abs(s["t"] - 0.5 * (t_start[k] + t_end[k])))] if samples else []
        r = {"step": k, "ms": float(dur[k]), "n_samples": len(ss),
             "kernel_mhz": float(100.0 * st[k, 0] / st[k, 1]) if cs is not None and st[k, 1] else None}
        for key in keys:
            v = [s[key] for s in ss if s.get(key) is not None]
            r[key] = float(np.mean(v)) if v else None
        rows.append(r)
    summary = {}
    for w in args.windows.split(","):
        a, b = (int(x) for x in w.split("-"))
        sel = [r for r in rows if a <= r["step"] <= b]
        summary[w] = {"ms_mean": float(np.mean([r["ms"] for r in sel]))}
        km = [r["kernel_mhz"] for r in sel if r["kernel_mhz"]]
        summary[w]["kernel_mhz"] = float(np.mean(km)) if km else None
        for key in keys:
            v = [r[key] for r in sel if r[key] is not None]
            summary[w][key] = float(np.mean(v)) if v else None
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"sysfs": base, "hwmon": hw, "files": {k: v[1] for k, v in files.items()}, "warmup": args.warmup,
                   "steps": rows, "windows": summary, "n_samples": len(samples),
                   "sample_period_ms": args.period}, f, indent=1)
    print(json.dumps(summary))
    for r in rows:
        print(r["step"], "%.1f us" % (1e3 * r["ms"]), "kernel_mhz=%s" % r["kernel_mhz"],
              " ".join(f"{k}={r[k]}" for k in keys))


if __name__ == "__main__":
    main()
