"""Timing experiments on the phase kernels WITHOUT touching the product
sources: copies csrc/ to a scratch dir, applies one named source edit, and
builds lib/exp/<name>/libdbsde.so (run it with DBSDE_LIB=<path>).  The
variants break the numerics on purpose -- timing only.

  nostore   every bstore() in phase.hpp is dropped (activation traffic out)
  noload    every bload() in phase.hpp returns zeros (activation reads out)
  nostage   each pass streams its first weight piece once, then reuses it
            without DMA or barriers (weight staging out)
  bare      nostore + noload + nostage

    python tools/exp_phase.py nostore noload nostage bare
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-neural-network-solutions-for-partial-differential-equations_amd")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC"]


def edit(src, name):
    if name in ("nostore", "bare"):
        src = src.replace("__device__ __forceinline__ void bstore(const Mat<TT>& m, float* base, int ld, int row0, int col0) {",
                          "__device__ __forceinline__ void bstore(const Mat<TT>& m, float* base, int ld, int row0, int col0) {\n"
                          "  if (ld > 0) return;")
    if name in ("noload", "bare"):
        src = src.replace("__device__ __forceinline__ void bload(Mat<TT>& m, const float* base, int ld, int row0, int col0) {",
                          "__device__ __forceinline__ void bload(Mat<TT>& m, const float* base, int ld, int row0, int col0) {\n"
                          "  if (ld > 0) { for (int t = 0; t < TT; ++t) m.v[t] = floatx4{0.f, 0.f, 0.f, 0.f}; return; }")
    if name in ("nostage", "bare"):
        src = src.replace("  __device__ __forceinline__ const floatx4* next() {\n",
                          "  __device__ __forceinline__ const floatx4* next() {\n"
                          "    if (st++ > 0) return wl;\n    vm_wait0();\n    __syncthreads();\n    return wl;\n")
    return src


def build(name):
    out = os.path.join(PKG, "lib", "exp", name)
    tmp = os.path.join("/tmp", "dbsde_exp_" + name)
    shutil.rmtree(tmp, ignore_errors=True)
    csrc = os.path.join(tmp, "pkg", "csrc")          # csrc/../../include resolves to tmp/include
    shutil.copytree(os.path.join(PKG, "csrc"), csrc)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    ph = os.path.join(csrc, "phase.hpp")
    s = open(ph).read()
    s2 = edit(s, name)
    assert s2 != s, name
    open(ph, "w").write(s2)
    os.makedirs(out, exist_ok=True)
    objs = []
    for unit, extra in (("engine.hip", []), ("evals.hip", []), ("tnw.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form=true"])):
        o = os.path.join(tmp, unit + ".o")
        subprocess.run([HIPCC, *FLAGS, *extra, "-c", "-o", o, os.path.join(csrc, unit)], check=True)
        objs.append(o)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libdbsde.so"), *objs],
                   check=True)
    print(os.path.join(out, "libdbsde.so"))


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
