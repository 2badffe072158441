import csv, glob, sys, collections
# usage: pmcsum.py tag kernel_substr
tag, ks = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if ks in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    # per dispatch sums are already per kernel dispatch; print mean over dispatches
    print(f"{k:28s} {sum(v)/len(v):.4g}  (n={len(v)})")
