"""rocprofv3 kernel-trace -> the per-step kernel timeline of bench.py's timed
steps: for a few steps, every launch's start / end offset (us) from the
step's first launch (rtr_params_kernel) and its queue, plus the median
offsets per kernel position over all timed steps (gaps and overlaps).

    python tools/timeline.py <run_kernel_trace.csv> [n_print] [out.txt]
"""
import csv
import sys
from collections import defaultdict

import numpy as np

SHORT = [("phaseA", "A"), ("phaseC", "C"), ("tnw_x3", "tnw"), ("tilefin", "fin"), ("proj_backward", "projb"),
         ("rtr_params", "rtr"), ("pack_tagged", "pack"), ("rollout", "roll"), ("optim", "opt"), ("sqnorm", "sq")]


def short(n):
    for k, v in SHORT:
        if k in n:
            return v
    return n.split("(")[0][-24:]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nprint = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows)
    # steps start at rtr_params_kernel
    steps, cur = [], None
    for e in ev:
        if e[2] == "rtr":
            if cur:
                steps.append(cur)
            cur = [e]
        elif cur is not None:
            cur.append(e)
    if cur:
        steps.append(cur)
    # timed steps: those with piped weight-gradient slices (tnw before the last C)
    def piped(st):
        names = [x[2] for x in st]
        return "tnw" in names and "C" in names and names.index("tnw") < len(names) - 1 - names[::-1].index("C")
    timed = [s for s in steps if piped(s)]
    lines = [f"{len(steps)} steps, {len(timed)} with piped weight-gradient slices"]
    for st in timed[2:2 + nprint]:
        t0 = st[0][0]
        lines.append("step:")
        for s, e, n, q in st:
            lines.append(f"  {n:8s} q{q:>3s} {1e-3 * (s - t0):8.1f} -> {1e-3 * (e - t0):8.1f}  ({1e-3 * (e - s):6.1f} us)")
    # median per (position, name)
    pos = defaultdict(list)
    for st in timed[1:]:
        t0 = st[0][0]
        nxt = None
        for i, (s, e, n, q) in enumerate(st):
            pos[(i, n)].append((1e-3 * (s - t0), 1e-3 * (e - t0)))
    lines.append("median offsets over timed steps (position, kernel, start, end, dur):")
    for (i, n), v in sorted(pos.items()):
        a = np.array(v)
        lines.append(f"  {i:2d} {n:8s} {np.median(a[:, 0]):8.1f} {np.median(a[:, 1]):8.1f} {np.median(a[:, 1] - a[:, 0]):7.1f}  n={len(v)}")
    spans = [1e-3 * (st[-1][1] - st[0][0]) for st in timed[1:]]
    starts = [1e-3 * (b[0][0] - a[0][0]) for a, b in zip(timed[1:], timed[2:])]
    lines.append(f"step span median {np.median(spans):.1f} us, step start-to-start median {np.median(starts):.1f} us")
    txt = "\n".join(lines)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
