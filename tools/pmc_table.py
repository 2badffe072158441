"""Per-kernel counter table of one profile directory (tools/profile_round.sh):
mean per dispatch of every counter, plus derived MFMA busy, wait shares and
HBM bytes (FETCH_SIZE doubled, MI355X_MICROARCH.md HBM section).
    python tools/pmc_table.py gpurun_out/prof_r4_bsb [kernel_substr ...]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
keys = sys.argv[2:] or ["phaseA", "phaseC", "tnw", "tn_x3", "rollout", "tilefin", "proj_backward", "pack", "rtr",
                        "optim", "chain"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = next((k for k in keys if k in name), None)
        if k is None:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
stats = {}
sf = glob.glob(os.path.join(d, "stats", "*kernel_stats.csv"))
if sf:
    for r in csv.DictReader(open(sf[0])):
        k = next((k for k in keys if k in r["Name"]), None)
        if k:
            s = stats.setdefault(k, [0, 0.0])
            s[0] += int(r["Calls"])
            s[1] += float(r["TotalDurationNs"])
for k in keys:
    c = {n: sum(v) / len(v) for n, v in agg[k].items()}
    if not c:
        continue
    out = [f"{k:14s}"]
    if k in stats:
        out.append(f"avg {stats[k][1] / stats[k][0] / 1e3:8.1f} us x{stats[k][0]}")
    g = c.get("GRBM_GUI_ACTIVE")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and g:
        out.append(f"mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (g / 8):.3f}")
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if n in c:
                out.append(f"{n[3:].lower()} {c[n] / w:.3f}")
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_MFMA" in c:
        out.append(f"valu/mfma {c['SQ_INSTS_VALU'] / max(c['SQ_INSTS_MFMA'], 1):.2f}")
    for n in ("SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT",
              "SQ_WAIT_INST_LDS"):
        if n in c:
            out.append(f"{n[3:].lower()} {c[n]:.3g}")
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out.append(f"hbm_MB {(2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024 / 1e6:.1f} "
                   f"(rd {2 * c['FETCH_SIZE'] * 1024 / 1e6:.1f} wr {c['WRITE_SIZE'] * 1024 / 1e6:.1f})")
    print("  ".join(out))
