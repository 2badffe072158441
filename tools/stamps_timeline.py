"""Timeline of the phase kernels from gpurun_out/stamps4.npy (tools/exp_phase.py
stamps4 + tools/stamps_dump.py): per launch (A0, C0, A1, C1) start spread,
lifetime, piece vmcnt / barrier waits; co-residency classes (what else ran on
the same CU during a workgroup's life).  Only the latest step is kept (a later
smaller launch may have overwritten some slots).

    python tools/stamps_timeline.py gpurun_out/stamps4.npy
"""
import collections
import statistics as st
import sys

import numpy as np

a = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps4.npy").astype(np.int64)
names = ["A0", "C0", "A1", "C1"]
recs = []
for k in range(4):
    for wg in range(a.shape[1]):
        w = a[k, wg, 0]
        if w[7] != 1:
            continue
        hw, xcc = int(w[0]), int(w[1]) & 15
        recs.append(dict(k=names[k], wg=wg, xcc=xcc, cu=(xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15),
                         s=int(w[2]), e=int(w[3]), vm=int(a[k, wg, :, 4].mean()), bar=int(a[k, wg, :, 5].mean()),
                         dma=int(a[k, wg, :, 6].mean()) if a.shape[3] > 8 else 0,
                         aft=int(a[k, wg, :, 8].mean()) if a.shape[3] > 8 else 0,
                         reg=int(a[k, wg, :, 9].mean()) if a.shape[3] > 8 else 0))
# latest step per XCC: starts within 2M cycles of that XCC's latest start
last = collections.defaultdict(int)
for r in recs:
    last[r["xcc"]] = max(last[r["xcc"]], r["s"])
recs = [r for r in recs if r["s"] > last[r["xcc"]] - 900_000]
base = {}
for r in recs:
    base[r["xcc"]] = min(base.get(r["xcc"], r["s"]), r["s"])
for r in recs:
    r["s"] -= base[r["xcc"]]
    r["e"] -= base[r["xcc"]]
    r["life"] = r["e"] - r["s"]
for k in names:
    v = [r for r in recs if r["k"] == k]
    if not v:
        continue
    print("%s n=%3d start min/med/max %7d %7d %7d  end max %7d  life med %6d (min %6d max %6d)  vm %5d bar %5d dma %5d after %5d mfma-regions %6d" % (
        k, len(v), min(r["s"] for r in v), st.median(r["s"] for r in v), max(r["s"] for r in v), max(r["e"] for r in v),
        st.median(r["life"] for r in v), min(r["life"] for r in v), max(r["life"] for r in v),
        st.median(r["vm"] for r in v), st.median(r["bar"] for r in v), st.median(r["dma"] for r in v),
        st.median(r["aft"] for r in v), st.median(r["reg"] for r in v)))
print("span per XCC:", {x: max(r["e"] for r in recs if r["xcc"] == x) for x in sorted(base)})
bycu = collections.defaultdict(list)
for r in recs:
    bycu[r["cu"]].append(r)
print("CUs", len(bycu), "WGs per CU", sorted(collections.Counter(len(v) for v in bycu.values()).items()))
cls = collections.defaultdict(list)
for cu, v in bycu.items():
    for r in v:
        sh = collections.Counter()
        for o in v:
            if o is r:
                continue
            ov = min(r["e"], o["e"]) - max(r["s"], o["s"])
            if ov > 0:
                sh[o["k"][0]] += ov / r["life"]
        cls[(r["k"][0], round(sh["A"] * 2) / 2, round(sh["C"] * 2) / 2)].append(r["life"])
print("kernel, co-resident A share, C share: n, median life")
for k in sorted(cls):
    print("  ", k, len(cls[k]), int(st.median(cls[k])))
