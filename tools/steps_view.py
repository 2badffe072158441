"""Print one timed step of a rocprofv3 kernel trace (offsets in us from the
step's rtr_params_kernel) and the median gaps around the phase section.
    python tools/steps_view.py <run_kernel_trace.csv> [step_index]"""
import csv
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from timeline import short  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
k0 = int(sys.argv[2]) if len(sys.argv) > 2 else 12
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
st = [i for i, e in enumerate(ev) if e[2] == "rtr"]
t0 = ev[st[k0]][0]
for s, e, n, q in ev[st[k0]:st[k0 + 1]]:
    print(f"  {n:10s} q{q} {1e-3 * (s - t0):8.1f} {1e-3 * (e - t0):8.1f} {1e-3 * (e - s):7.1f}")
span = [(ev[st[k + 1]][0] - ev[st[k]][0]) / 1e3 for k in range(5, len(st) - 1)]
print("step median", np.median(span), "us over", len(span))
