"""Timing experiments on the phase kernels WITHOUT touching the product
sources: copies csrc/ to a scratch dir, applies one named source edit, and
builds lib/exp/<name>/libdbsde.so (run it with DBSDE_LIB=<path>).  The
variants break the numerics on purpose -- timing only.

  nostore   every bstore() in phase.hpp is dropped (activation traffic out)
  noload    every bload() in phase.hpp returns zeros (activation reads out)
  nostage   each pass streams its first weight piece once, then reuses it
            without DMA or barriers (weight staging out)
  bare      nostore + noload + nostage
  ntstore   bstore() uses nontemporal stores (streaming, no L2 allocate)
  ntload    bload() uses nontemporal loads
  ntsel     nontemporal stores only for arrays the weight-gradient kernel reads
            (H, Delta, Hdot, Alpha, zbar); Abuf/G/zfull (read by phase C) cached
  ntsel2    the complement of ntsel
  noslp     -fno-slp-vectorize (no v_pk_* f32 packing)
  tnwhit    weight-gradient x3 kernel loading one fixed 32-row block (cache hits)
  nostoreall / noloadall / bareall  every activation store / load / both, + nostage
  stamps    -DDBSDE_STAMPS: per-piece s_memtime (wait / MFMA issue / post)
            printed for three tiles -- diagnostic only
  quadplain quad-order stores of the weight-gradient operands without the
            nontemporal hint

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
    if name in ("ntstore", "ntboth"):
        src = src.replace("  for (int t = 0; t < TT; ++t) *(floatx4*)(p + 16 * t) = m.v[t];",
                          "  for (int t = 0; t < TT; ++t) __builtin_nontemporal_store(m.v[t], (floatx4*)(p + 16 * t));")
    if name in ("ntload", "ntboth"):
        src = src.replace("  for (int t = 0; t < TT; ++t) m.v[t] = *(const floatx4*)(p + 16 * t);",
                          "  for (int t = 0; t < TT; ++t) m.v[t] = __builtin_nontemporal_load((const floatx4*)(p + 16 * t));")
    if name == "quadplain":
        src = src.replace("    for (int t = 0; t < TT; ++t) __builtin_nontemporal_store(m.v[t], (floatx4*)(p + 64 * t));",
                          "    for (int t = 0; t < TT; ++t) *(floatx4*)(p + 64 * t) = m.v[t];")
    if name == "allplain":
        src = src.replace("__builtin_nontemporal_store(m.v[t], (floatx4*)(p + 64 * t));", "*(floatx4*)(p + 64 * t) = m.v[t];")
        src = src.replace("__builtin_nontemporal_store(m.v[t], (floatx4*)(p + 16 * t));", "*(floatx4*)(p + 16 * t) = m.v[t];")
    if name in ("ntsel", "ntsel2"):
        nt_arrays = ("p.H,", "p.Delta,", "p.Hdot,", "p.Alpha,", "p.zbar,")
        if name == "ntsel2":
            nt_arrays = ("p.Abuf,", "p.G,", "p.zfull,")
        src = src.replace("__device__ __forceinline__ void bstore(const Mat<TT>& m, float* base, int ld, int row0, int col0) {",
                          "__device__ __forceinline__ void bstore_nt(const Mat<TT>& m, float* base, int ld, int row0, int col0) {\n"
                          "  const int lane = threadIdx.x & 63;\n"
                          "  float* p = base + (size_t)(row0 + (lane & 15)) * ld + col0 + 4 * (lane >> 4);\n"
                          "#pragma unroll\n"
                          "  for (int t = 0; t < TT; ++t) __builtin_nontemporal_store(m.v[t], (floatx4*)(p + 16 * t));\n}\n"
                          "template <int TT>\n"
                          "__device__ __forceinline__ void bstore(const Mat<TT>& m, float* base, int ld, int row0, int col0) {")
        lines = src.split("\n")
        for i, ln in enumerate(lines):
            if "bstore(" in ln and "void bstore" not in ln and any(a in ln for a in nt_arrays):
                lines[i] = ln.replace("bstore(", "bstore_nt(")
        src = "\n".join(lines)
    if name in ("nostoreall", "bareall"):   # every activation store (bstore, fstore, streaming) dropped
        for fn in ("bstore", "fstore", "bstore_stream"):
            sig = "__device__ __forceinline__ void %s(const Mat<TT>& m, float* base, int ld, int row0, int col0) {" % fn
            assert sig in src, fn
            src = src.replace(sig, sig + "\n  if (ld > 0) return;")
    if name in ("noloadall", "bareall"):    # every activation load (bload, fload) returns zeros
        for fn in ("bload", "fload"):
            sig = "__device__ __forceinline__ void %s(Mat<TT>& m, const float* base, int ld, int row0, int col0) {" % fn
            assert sig in src, fn
            src = src.replace(sig, sig + "\n  if (ld > 0) { for (int t = 0; t < TT; ++t) m.v[t] = floatx4{0.f, 0.f, 0.f, 0.f}; return; }")
    if name in ("stamps2", "stamps3"):   # per-wave s_memtime sums: piece vmcnt wait, barrier wait, kernel total (printf)
        a = "  __device__ __forceinline__ const floatx4* next() {\n"
        assert a in src
        src = src.replace("  int n, st, wave, lane, buf;\n", "  int n, st, wave, lane, buf;\n  unsigned long long tvm = 0, tbar = 0;\n")
        src = src.replace("      wait_younger<NYOUNG, NBUF - 2>(k);\n    } else {\n      vm_wait<NYOUNG>();\n    }\n    lds_barrier();\n",
                          "      const unsigned long long ta = __builtin_amdgcn_s_memtime();\n      wait_younger<NYOUNG, NBUF - 2>(k);\n"
                          "      const unsigned long long tb = __builtin_amdgcn_s_memtime();\n      lds_barrier();\n"
                          "      const unsigned long long tc = __builtin_amdgcn_s_memtime();\n      tvm += tb - ta; tbar += tc - tb;\n"
                          "    } else {\n      vm_wait<NYOUNG>();\n      lds_barrier();\n    }\n")
        for kern, tag in (("phaseA_kernel(FusedArgs p) {\n", "A"), ("phaseC_kernel(FusedArgs p) {\n", "C")):
            i = src.index(kern) + len(kern)
            src = src[:i] + "  const unsigned long long t_start = __builtin_amdgcn_s_memtime();\n" + src[i:]
        # kernel ends: the closing brace before the phase C comment / the namespace end
        endA = src.index("// phase C: cotangents")
        j = src.rindex("}\n", 0, endA)
        sel = "(blockIdx.x % 50) == 0" if name == "stamps2" else "threadIdx.x == 0"
        src = src[:j] + ('  if ((threadIdx.x & 63) == 0 && ' + sel + ') printf("STAMP A tile0=%d wg=%d wave=%d hw=%u xcc=%u t0=%llu total=%llu vm=%llu bar=%llu\\n", p.tile0, (int)blockIdx.x, wave, __builtin_amdgcn_s_getreg(63492), __builtin_amdgcn_s_getreg(63508), t_start, __builtin_amdgcn_s_memtime() - t_start, sg.tvm, sg.tbar);\n') + src[j:]
        endC = src.index("}  // namespace dbsde")
        j = src.rindex("}\n", 0, endC)
        src = src[:j] + ('  if ((threadIdx.x & 63) == 0 && ' + sel + ') printf("STAMP C tile0=%d wg=%d wave=%d hw=%u xcc=%u t0=%llu total=%llu vm=%llu bar=%llu\\n", p.tile0, (int)blockIdx.x, wave, __builtin_amdgcn_s_getreg(63492), __builtin_amdgcn_s_getreg(63508), t_start, __builtin_amdgcn_s_memtime() - t_start, sg.tvm, sg.tbar);\n') + src[j:]
    if name in ("stamps4", "stamps5"):   # per-workgroup stamps into a device array (no printf): tools/stamps_dump.py reads it
        src = src.replace("  int n, st, wave, lane, buf;\n", "  int n, st, wave, lane, buf;\n  unsigned long long tvm = 0, tbar = 0;\n")
        src = src.replace("      wait_younger<NYOUNG, NBUF - 2>(k);\n    } else {\n      vm_wait<NYOUNG>();\n    }\n    lds_barrier();\n",
                          "      const unsigned long long ta = __builtin_amdgcn_s_memtime();\n      wait_younger<NYOUNG, NBUF - 2>(k);\n"
                          "      const unsigned long long tb = __builtin_amdgcn_s_memtime();\n      lds_barrier();\n"
                          "      const unsigned long long tc = __builtin_amdgcn_s_memtime();\n      tvm += tb - ta; tbar += tc - tb;\n"
                          "    } else {\n      vm_wait<NYOUNG>();\n      lds_barrier();\n    }\n")
        src = src.replace("namespace dbsde {\n\nconstexpr int P3_WAVES = 4;",
                          "namespace dbsde {\n\n__device__ unsigned long long g_stamps[4 * 1024 * 32];\nconstexpr int P3_WAVES = 4;")
        for kern in ("phaseA_kernel(FusedArgs p) {\n", "phaseC_kernel(FusedArgs p) {\n"):
            i = src.index(kern) + len(kern)
            src = src[:i] + "  const unsigned long long t_start = __builtin_amdgcn_s_memtime();\n" + src[i:]
        rec = ('  if ((threadIdx.x & 63) == 0) {{ unsigned long long* g = g_stamps + (({isc} + 2 * (p.tile0 != 0)) * 1024 + blockIdx.x) * 32 + wave * 8;'
               ' g[0] = __builtin_amdgcn_s_getreg(63492); g[1] = __builtin_amdgcn_s_getreg(63508); g[2] = t_start;'
               ' g[3] = __builtin_amdgcn_s_memtime(); g[4] = sg.tvm; g[5] = sg.tbar; g[6] = blockIdx.x; g[7] = 1; }}\n')
        endA = src.index("// phase C: cotangents")
        j = src.rindex("}\n", 0, endA)
        src = src[:j] + rec.format(isc=0) + src[j:]
        endC = src.index("}  // namespace dbsde")
        j = src.rindex("}\n", 0, endC)
        src = src[:j] + rec.format(isc=1) + src[j:]
    if name == "stamps5":   # stamps4 + per-category sums: DMA issue, after() (stores / loads), MFMA regions
        src = src.replace("  unsigned long long tvm = 0, tbar = 0;\n", "")
        src = src.replace("  int n, st, wave, lane, buf;\n", "  int n, st, wave, lane, buf;\n  unsigned long long tvm = 0, tbar = 0, tdma = 0, taft = 0, treg = 0;\n", 1)
        a = "    if (st + DIST < n) piece_dma(img[st + DIST], nf[st + DIST], wl + ((st + DIST) % NBUF) * buf, wave, lane);\n"
        assert a in src
        src = src.replace(a, "    const unsigned long long td0 = __builtin_amdgcn_s_memtime();\n" + a +
                          "    tdma += __builtin_amdgcn_s_memtime() - td0;\n")
        a = "    if constexpr (KB == 0) {\n      after();\n"
        assert a in src
        src = src.replace(a, "    if constexpr (KB == 0) {\n      const unsigned long long ta0 = __builtin_amdgcn_s_memtime();\n      after();\n"
                          "      sg.taft += __builtin_amdgcn_s_memtime() - ta0;\n")
        a = "    sgemm_x3_piece<TO, TI, KB + 1, PF>(acc, s, w, lane, b, sn);\n"
        assert a in src
        src = src.replace(a, "    const unsigned long long tr0 = __builtin_amdgcn_s_memtime();\n" + a +
                          "    sg.treg += __builtin_amdgcn_s_memtime() - tr0;\n")
        src = src.replace("g[6] = blockIdx.x; g[7] = 1; }", "g[6] = sg.tdma; g[7] = 1; g[8] = sg.taft; g[9] = sg.treg; }")
        src = src.replace("* 32 + wave * 8;", "* 64 + wave * 16;")
        src = src.replace("g_stamps[4 * 1024 * 32]", "g_stamps[4 * 1024 * 64]")
    if name in ("nostage", "bare", "bareall"):
        src = src.replace("  __device__ __forceinline__ const floatx4* next() {\n",
                          "  __device__ __forceinline__ const floatx4* next() {\n"
                          "    if (st++ > 0) return wl;\n    vm_wait<0>();\n    __syncthreads();\n    return wl;\n")
    return src


def build(name):
    out = os.path.join(PKG, "lib", "exp", name)
    tmp = os.path.join("/tmp", "dbsde_exp_" + name)
    shutil.rmtree(tmp, ignore_errors=True)
    csrc = os.path.join(tmp, "pkg", "csrc")          # csrc/../../include resolves to tmp/include
    shutil.copytree(os.path.join(PKG, "csrc"), csrc)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    if name == "tnwvec":   # weight-gradient x3 operand loads as 2 float4 per lane and block (wrong layout; timing only)
        tx = os.path.join(csrc, "tnwx3.hip")
        t = open(tx).read()
        a = ("  for (int j = 0; j < 8; ++j) {\n    const float* p = X + (size_t)(row0 + j) * ld + i;\n#pragma unroll\n"
             "    for (int m = 0; m < NB; ++m) r[m][j] = p[16 * m];\n  }")
        assert a in t, "tnwvec load_cols"
        t = t.replace(a, "  for (int m = 0; m < NB; ++m) {\n    const float* p = X + (size_t)(row0 + (i >> 1)) * ld + 16 * m + 8 * (i & 1);\n"
                         "    const floatx4 u = *(const floatx4*)p, v = *(const floatx4*)(p + 4);\n"
                         "    r[m][0] = u[0]; r[m][1] = u[1]; r[m][2] = u[2]; r[m][3] = u[3];\n"
                         "    r[m][4] = v[0]; r[m][5] = v[1]; r[m][6] = v[2]; r[m][7] = v[3];\n  }")
        b = "    for (int j = 0; j < 8; ++j) ra[0][j] = A[(size_t)(nrow + j) * lda + i];"
        assert b in t, "tnwvec a0"
        t = t.replace(b, "    for (int jj = 0; jj < 1; ++jj) { const float* q4 = A + (size_t)(nrow + (i >> 1)) * lda + 8 * (i & 1); const floatx4 u = *(const floatx4*)q4, v = *(const floatx4*)(q4 + 4);"
                         " ra[0][0] = u[0]; ra[0][1] = u[1]; ra[0][2] = u[2]; ra[0][3] = u[3]; ra[0][4] = v[0]; ra[0][5] = v[1]; ra[0][6] = v[2]; ra[0][7] = v[3]; }")
        c = "        for (int j = 0; j < 8; ++j) ra[m + 1][j] = A[(size_t)(nrow + j) * lda + 16 * (m + 1) + i];"
        assert c in t, "tnwvec am"
        t = t.replace(c, "        for (int jj = 0; jj < 1; ++jj) { const float* q4 = A + (size_t)(nrow + (i >> 1)) * lda + 16 * (m + 1) + 8 * (i & 1); const floatx4 u = *(const floatx4*)q4, v = *(const floatx4*)(q4 + 4);"
                         " ra[m + 1][0] = u[0]; ra[m + 1][1] = u[1]; ra[m + 1][2] = u[2]; ra[m + 1][3] = u[3]; ra[m + 1][4] = v[0]; ra[m + 1][5] = v[1]; ra[m + 1][6] = v[2]; ra[m + 1][7] = v[3]; }")
        open(tx, "w").write(t)
    if name == "tnwhit":   # weight-gradient x3 operand loads from a fixed 32-row block (cache hits)
        tx = os.path.join(csrc, "tnwx3.hip")
        t = open(tx).read()
        t2 = t.replace("const float* p = X + (size_t)(row0 + j) * ld + i;", "const float* p = X + (size_t)(j + 8 * (row0 & 31) / 8) * ld + i;")
        t2 = t2.replace("ra[m + 1][j] = A[(size_t)(nrow + j) * lda", "ra[m + 1][j] = A[(size_t)(j + (nrow & 31)) * lda")
        t2 = t2.replace("ra[0][j] = A[(size_t)(nrow + j) * lda", "ra[0][j] = A[(size_t)(j + (nrow & 31)) * lda")
        assert t2.count("nrow & 31") == 2, "tnwhit edit"
        open(tx, "w").write(t2)
    ph = os.path.join(csrc, "phase.hpp")
    s = open(ph).read()
    defs = []
    eng_edits = {   # engine.hip launch-shape variants
        "onechunk": ("  int chunks = 2;", "  int chunks = 1;"),    # all of phase A, then all of phase C
        "onepipe": ("  int pipes = 2;", "  int pipes = 1;"),       # A0 C0 A1 C1 in order on one stream
        # unequal path chunks (units of 64 paths; 16 at the north star)
        "c0_6": ("  int chunk0 = 0;", "  int chunk0 = 6;"),
        "c0_7": ("  int chunk0 = 0;", "  int chunk0 = 7;"),
        "c0_9": ("  int chunk0 = 0;", "  int chunk0 = 9;"),
        "c0_10": ("  int chunk0 = 0;", "  int chunk0 = 10;"),
    }
    if name in eng_edits:
        ep = os.path.join(csrc, "engine.hip")
        e = open(ep).read()
        a, b = eng_edits[name]
        assert a in e, name
        open(ep, "w").write(e.replace(a, b))
    if name in ("stamps4", "stamps5"):   # the host-side reader of g_stamps
        ep = os.path.join(csrc, "engine.hip")
        e = open(ep).read()
        e += ('\nextern "C" int dbsde_exp_stamps(unsigned long long* out, long long n) {\n'
              '  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dbsde::g_stamps), n * 8, 0, hipMemcpyDeviceToHost);\n}\n')
        open(ep, "w").write(e)
    file_edits = {   # timing-only ablations of the phase kernels' instruction classes
        # no LDS fragment reads in the split-bf16 pieces (register constants as weights)
        "nolds": [("phase.hpp", "w[(o + 1) & 1][p] = im[(3 * (o + 1) + p) * 64 + lane];",
                   "w[(o + 1) & 1][p] = uintx4{(unsigned)lane, (unsigned)p, 7u, (unsigned)o};"),
                  ("phase.hpp", "for (int p = 0; p < 3; ++p) w[0][p] = im[p * 64 + lane];",
                   "for (int p = 0; p < 3; ++p) w[0][p] = uintx4{(unsigned)lane, (unsigned)p, 7u, 3u};"),
                  ("phase.hpp", "for (int p = 0; p < 3; ++p) w[0][p] = im[(3 * o + p) * 64 + lane];",
                   "for (int p = 0; p < 3; ++p) w[0][p] = uintx4{(unsigned)lane, (unsigned)p, 7u, (unsigned)o};")],
        # no activation split: hi = x0 bits, mid = x1 bits, lo = 0 (0 VALU)
        "nosplit": [("phase.hpp", "__device__ __forceinline__ Dw3 split_two(float x0, float x1) {",
                     "__device__ __forceinline__ Dw3 split_two(float x0, float x1) {\n"
                     "  if (x0 != 12345.f) return Dw3{__float_as_uint(x0), __float_as_uint(x1), 0u};")],
        # no transcendental activation: sin -> a, cos -> 1
        "noact": [("kernels.hpp", "__device__ __forceinline__ void fast_sincosf(float a, float& s, float& c) {",
                   "__device__ __forceinline__ void fast_sincosf(float a, float& s, float& c) {\n"
                   "  if (a != 12345.f) { s = a; c = 1.f; return; }")],
        # fewer products per split-bf16 fragment (MFMA-pipe sensitivity; wrong numerics)
        "mfma3": [("phase.hpp", "    a = mfma_bf(wc[0], s.l, a);\n    a = mfma_bf(wc[0], s.m, a);\n    a = mfma_bf(wc[1], s.m, a);\n", "")],
        "mfma1": [("phase.hpp", "    a = mfma_bf(wc[0], s.l, a);\n    a = mfma_bf(wc[0], s.m, a);\n    a = mfma_bf(wc[1], s.m, a);\n"
                   "    a = mfma_bf(wc[1], s.h, a);\n    a = mfma_bf(wc[2], s.h, a);\n", "")],
        # no pinned MFMA / VALU interleave in the split-bf16 pieces
        "nosched": [("phase.hpp", "      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA\n"
                                  "      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU\n", "")],
    }
    if name in file_edits:
        for fn, a, b in file_edits[name]:
            fp = os.path.join(csrc, fn)
            t = open(fp).read()
            assert a in t, (name, a[:60])
            open(fp, "w").write(t.replace(a, b))
    elif name in eng_edits:
        pass
    elif name == "stamps":    # per-piece s_memtime printf of three tiles (diagnostic build)
        defs = ["-DDBSDE_STAMPS"]
    elif name == "noslp":   # no SLP packing of f32 elementwise work into v_pk_* (MI355X_MICROARCH: anti-lever beside MFMA)
        defs = ["-fno-slp-vectorize"]
    elif name in ("tnwhit", "tnwvec"):
        pass
    else:
        s2 = edit(s, name)
        assert s2 != s, name
        open(ph, "w").write(s2)
    os.makedirs(out, exist_ok=True)
    objs = []
    sys.path.insert(0, PKG)
    from build_lib import UNITS
    for unit, extra in UNITS:
        o = os.path.join(tmp, unit + ".o")
        subprocess.run([HIPCC, *FLAGS, *extra, *defs, "-c", "-o", o, os.path.join(csrc, unit)], check=True)
        objs.append(o)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libdbsde.so"), *objs],
                   check=True)
    print(os.path.join(out, "libdbsde.so"))


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
