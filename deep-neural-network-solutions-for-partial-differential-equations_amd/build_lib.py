"""Build lib/libdbsde.so from csrc/ with hipcc for gfx950 (in-tree, so the
shared object travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
# translation units and their extra flags: the weight-gradient kernel is built
# with VGPR-form MFMA (see csrc/tnw.hip); everything else (its split-bf16 form
# tnwx3.hip included: accumulators in AGPRs) with the defaults
UNITS = [("engine.hip", []), ("phase2.hip", []), ("phasecs.hip", []), ("evals.hip", []), ("tnw.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form=true"]),
         ("tnwx3.hip", [])]
DEPS = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".hpp"))] + \
    [os.path.join(ROOT, "include", "dbsde.h")]
OUT = os.path.join(HERE, "lib", "libdbsde.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall"]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in DEPS)


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    objdir = os.path.join(HERE, "lib", "obj")
    os.makedirs(objdir, exist_ok=True)
    cmds, objs = [], []
    for src, extra in UNITS:
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        cmds.append([HIPCC, *FLAGS, *extra, "-c", "-o", obj, os.path.join(CSRC, src)])
        objs.append(obj)
    procs = []
    for cmd in cmds:                       # the units compile in parallel
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    failed = False
    for p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out)
            failed = True
    if failed:
        raise RuntimeError("hipcc failed building libdbsde.so")
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(link), flush=True)
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed linking libdbsde.so")
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
