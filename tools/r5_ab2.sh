#!/bin/bash
# A/B after giving each used stream its own hardware queue: 2 vs 3 vs 4 chunks (bsb, basket)
export TMPDIR=/tmp
out=gpurun_out/r5ab2
mkdir -p $out
run() {  # run <tag> <env> <extra>
  env $2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity $3 > $out/$1.json 2>/dev/null || { echo "$1 failed"; exit 1; }
  python -c "import json;d=json.load(open('$out/$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],4))"
}
for rep in 1 2; do
  run base$rep "X=0" "--steps 100 --warmup 50"
  run ch3_$rep "DBSDE_CHUNKS=3" "--steps 100 --warmup 50"
  run ch4_$rep "DBSDE_CHUNKS=4" "--steps 100 --warmup 50"
  run bask$rep "X=0" "--steps 30 --warmup 10 --workload basket"
  run bask4_$rep "DBSDE_CHUNKS=4" "--steps 30 --warmup 10 --workload basket"
  run bask8_$rep "DBSDE_CHUNKS=8" "--steps 30 --warmup 10 --workload basket"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > $out/tr.log 2>&1 || exit 1
python - <<'PY'
import csv, sys, glob
import numpy as np
sys.path.insert(0,'tools')
from timeline import short
f=glob.glob('gpurun_out/r5ab2/tr/**/run_kernel_trace.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
ev=sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
st=[i for i,e in enumerate(ev) if e[2]=='rtr']
for k in (12,):
    t0=ev[st[k]][0]
    for s,e,n,q in ev[st[k]:st[k+1]]:
        print(f"  {n:10s} q{q} {1e-3*(s-t0):8.1f} {1e-3*(e-t0):8.1f} {1e-3*(e-s):7.1f}")
g1=[];g2=[];g3=[];span=[]
for k in range(5,len(st)-1):
    seg=ev[st[k]:st[k+1]]
    d={}
    for s,e,n,q in seg: d.setdefault(n,[]).append((s,e,q))
    if 'A' not in d or 'fin' not in d or 'tnw' not in d: continue
    g1.append((min(x[0] for x in d['A'])-d['pack'][0][1])/1e3); g2.append((d['fin'][0][0]-max(x[1] for x in d['tnw']))/1e3)
    g3.append((ev[st[k+1]][0]-d['projb'][0][1])/1e3); span.append((ev[st[k+1]][0]-ev[st[k]][0])/1e3)
print('pack->A0', np.median(g1), 'tnw->fin', np.median(g2), 'projb->next rtr', np.median(g3), 'step', np.median(span), len(span))
PY
