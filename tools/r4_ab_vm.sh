#!/bin/bash
# GPU parity of the new kernel forms, then A/Bs: piece vmcnt counts (vm0 =
# earlier counts), weight-gradient MFMA order (tnwchain = dependent chains);
# strong-scaling shapes: column-split (default at M <= 256) vs 64-row kernels
export TMPDIR=/tmp
mkdir -p gpurun_out/ablib
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_round4.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ablib/tests.txt 2>&1
rc=$?; tail -15 gpurun_out/ablib/tests.txt; [ $rc -le 1 ] || exit $rc
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:9]})
PY
}
for m in 128 256 512; do
  for v in "X=1" "DBSDE_CS=0" "DBSDE_CS=1 DBSDE_CHUNKS=1"; do
    tag=$(echo "$v" | tr ' =' '__')
    env $v timeout -k 10 200 python bench.py --paths-per-gpu $m --no-cpu-baseline --no-parity --steps 100 > gpurun_out/ablib/m${m}_$tag.log 2>&1 || { echo fail m$m $v; tail -5 gpurun_out/ablib/m${m}_$tag.log; exit 1; }
    summ gpurun_out/ablib/m${m}_$tag.log "M=$m $v"
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 > gpurun_out/ablib/bsb_default.log 2>&1 && summ gpurun_out/ablib/bsb_default.log "bsb M=1024"
# column-split weight feed: registers (base) vs the shared LDS-DMA ring (csl)
tools/ab_libs.sh "--paths-per-gpu 128 --no-cpu-baseline --no-parity --steps 100" csl > gpurun_out/ablib/csl.txt 2>&1; cat gpurun_out/ablib/csl.txt
