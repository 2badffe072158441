"""rocprofv3 kernel-trace -> per-step spans, the trace-side counterpart of
bench.py's event records: `fused_phases_pipelined` = first phaseA start to
last phaseC end of each step (the two path chunks on two streams overlap, so
their per-kernel durations do not add up to the section).  In unprofiled
steps each chunk's weight-gradient slices run inside that span (engine.hip
tnw_piped), so the trace span of those steps is the phases plus the overlap.

    python tools/trace_sections.py <run_kernel_trace.csv> [out.json]
"""
import csv
import json
import sys

import numpy as np


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # per step: [phase start, last phase C end, closed, weight-gradient launch seen before the last phase C]
    steps, cur = [], None
    for s, e, n in ev:
        if "phaseA_kernel" in n:
            if cur is None or cur[2]:      # a new step's first phase-A launch
                if cur is not None:
                    steps.append(cur)
                cur = [s, e, False, False, None]
            cur[1] = max(cur[1], e)
        elif "phaseC_kernel" in n and cur is not None:
            cur[1] = max(cur[1], e)
            if cur[4] is not None:
                cur[3] = True
        elif "tnw" in n and cur is not None and not cur[2]:
            cur[4] = s
        elif ("tilefin_kernel" in n or "slabsum_kernel" in n) and cur is not None:
            cur[2] = True                  # the step's finalize: the next phase A opens a new step
    if cur is not None:
        steps.append(cur)
    steps = steps[1:]                      # drop the first (warm-up) step

    def stats(v):
        v = np.array(v, dtype=float) / 1e3
        return {"mean": float(v.mean()), "median": float(np.median(v)), "min": float(v.min()), "max": float(v.max()),
                "n": int(v.size)} if v.size else None

    out = {"fused_phases_pipelined_us": stats([c[1] - c[0] for c in steps if not c[3]]),
           "note": "steps whose weight-gradient launch follows the section (bench.py's profiled pass: the roofline's section)",
           "phases_with_piped_weight_grad_us": stats([c[1] - c[0] for c in steps if c[3]]),
           "note_piped": "timed steps: each chunk's weight-gradient slices run inside the span"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
