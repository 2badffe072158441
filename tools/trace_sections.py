"""rocprofv3 kernel-trace -> per-step spans, the trace-side counterpart of
bench.py's event records: `fused_phases_pipelined` = first phaseA start to
last phaseC end of each step (the two path chunks on two streams overlap, so
their per-kernel durations do not add up to the section).

    python tools/trace_sections.py <run_kernel_trace.csv> [out.json]
"""
import csv
import json
import sys

import numpy as np


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    spans, cur = [], None
    for s, e, n in ev:
        if "phaseA_kernel" in n:
            if cur is None or cur[2]:      # a new step's first phase-A launch
                if cur is not None:
                    spans.append(cur[1] - cur[0])
                cur = [s, e, False]
            cur[1] = max(cur[1], e)
        elif "phaseC_kernel" in n and cur is not None:
            cur[1] = max(cur[1], e)
        elif "tnw_kernel" in n and cur is not None:
            cur[2] = True                  # the section ends before the weight gradients
    if cur is not None:
        spans.append(cur[1] - cur[0])
    spans = np.array(spans[1:], dtype=float) / 1e3   # drop the first (warm-up) step
    out = {"fused_phases_pipelined_us": {"mean": float(spans.mean()), "median": float(np.median(spans)),
                                          "min": float(spans.min()), "max": float(spans.max()), "n": int(spans.size)}}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
