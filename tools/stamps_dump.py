"""Run bench.py's main() in-process with an exp "stamps4" library (DBSDE_LIB,
tools/exp_phase.py) and dump the per-workgroup phase-kernel stamps of the last
step to gpurun_out/stamps4.npy: [kernel (A0, C0, A1, C1)][wg][wave][hw_id,
xcc_id, t_start, t_end, vmcnt-wait, barrier-wait, wg, valid] (s_memtime cycles).

    DBSDE_LIB=.../lib/exp/stamps4/libdbsde.so python tools/stamps_dump.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
lib = ctypes.CDLL(os.environ["DBSDE_LIB"])
W = int(os.environ.get("STAMP_WORDS", "8"))   # 8 (stamps4) or 16 (stamps5)
n = 4 * 1024 * W * 4
buf = np.zeros(n, np.uint64)
rc = lib.dbsde_exp_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(n))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", "stamps4.npy"), buf.reshape(4, 1024, 4, W))
print("stamps rc", rc)
