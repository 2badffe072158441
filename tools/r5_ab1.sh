#!/bin/bash
# A/B: chunk stream assignment, prefetch, 4 chunks with the weight-gradient stream; host enqueue probe
export TMPDIR=/tmp
out=gpurun_out/r5ab1
mkdir -p $out
B="python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50"
run() {  # run <tag> <env> <extra>
  env $2 timeout -k 10 300 $B $3 > $out/$1.json 2>/dev/null || { echo "$1 failed"; exit 1; }
  python -c "import json;d=json.load(open('$out/$1.json'));print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],4))"
}
for rep in 1 2; do
  run base$rep "X=0" ""
  run swap$rep "DBSDE_CHUNK_SWAP=1" ""
  run nopf$rep "X=0" "--no-prefetch"
  run ch4_$rep "DBSDE_CHUNKS=4" ""
  run ch4swap$rep "DBSDE_CHUNKS=4 DBSDE_CHUNK_SWAP=1" ""
done
timeout -k 10 300 python tools/host_probe.py > $out/host.json 2>/dev/null && cat $out/host.json
timeout -k 10 300 python tools/host_probe.py --no-prefetch > $out/host_nopf.json 2>/dev/null && cat $out/host_nopf.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 --workload basket > $out/basket.json 2>/dev/null
DBSDE_CHUNKS=4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 --workload basket > $out/basket4.json 2>/dev/null
python -c "
import json
for f in ('basket','basket4'):
    d=json.load(open('$out/'+f+'.json')); print(f, round(d['value']/1e6,2), round(d['ms_per_step'],4))"
