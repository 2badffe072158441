"""The C-ABI library: builds, loads, exports every symbol include/dbsde.h
declares, and its struct layouts agree with the ctypes mirror.  No GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, load_pkg

HEADER = os.path.join(ROOT, "include", "dbsde.h")


@pytest.fixture(scope="module")
def lib():
    pkg = load_pkg()
    import importlib
    importlib.import_module(pkg.__name__ + ".build_lib").build(verbose=False)
    return pkg._lib.load()


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^[a-z][\w \*]*?\b(dbsde_\w+)\s*\(", txt, flags=re.M)))


def test_header_and_binding_agree():
    pkg = load_pkg()
    assert header_functions() == sorted(pkg._lib.EXPORTED)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", load_pkg()._lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dbsde_\w+)", out))
    missing = set(header_functions()) - exported
    assert not missing, missing
    for name in header_functions():
        assert hasattr(lib, name)


def test_abi_version_and_config_validation(lib):
    pkg = load_pkg()
    assert lib.dbsde_abi_version() == pkg._lib.ABI_VERSION == 3
    cfg = pkg._lib.Config()
    cfg.mode, cfg.activation, cfg.n_layers = 1, 0, 2          # too few layers -> EINVAL before any HIP call
    ctx = ctypes.c_void_p()
    rc = lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx))
    assert rc == pkg._lib.DBSDE_EINVAL and not ctx.value
    assert b"len(layers)" in lib.dbsde_last_error(None)
    with pytest.raises(ValueError):
        pkg._lib.check(rc)
    for k, v in enumerate([5, 16, 16, 16, 16, 1]):
        cfg.layers[k] = v
    cfg.n_layers, cfg.mode = 6, 9                               # unknown mode
    assert lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx)) == pkg._lib.DBSDE_EINVAL
    cfg.mode, cfg.n_layers = 2, 6
    cfg.layers[2] = 8                                           # residual widths must match
    assert lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx)) == pkg._lib.DBSDE_EINVAL
    assert lib.dbsde_param_count(None) == -1


C_PROBE = r'''
#include <stdio.h>
#include <stddef.h>
#include "dbsde.h"
#define F(T, m) printf(#T "." #m " %zu\n", offsetof(T, m));
int main(void) {
  printf("dbsde_problem %zu\ndbsde_config %zu\ndbsde_batch %zu\ndbsde_outputs %zu\ndbsde_optim %zu\n",
         sizeof(dbsde_problem), sizeof(dbsde_config), sizeof(dbsde_batch), sizeof(dbsde_outputs),
         sizeof(dbsde_optim));
  F(dbsde_config, problem) F(dbsde_config, T) F(dbsde_config, device)
  F(dbsde_batch, seed) F(dbsde_batch, path0) F(dbsde_batch, Xi) F(dbsde_batch, xi_rows)
  F(dbsde_optim, max_norm) F(dbsde_optim, step) F(dbsde_problem, q3)
  F(dbsde_problem, kind) F(dbsde_problem, g_cols) F(dbsde_problem, u_clamp) F(dbsde_problem, h_rho)
  F(dbsde_optim, alpha) F(dbsde_optim, asgd_mu) F(dbsde_optim, loss)
  F(dbsde_optim, step_state) F(dbsde_optim, step_parity)
  return 0;
}
'''


def test_struct_layouts_match_ctypes(tmp_path):
    pkg = load_pkg()
    src = tmp_path / "probe.c"
    src.write_text(C_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.split("\n") if line)
    L = pkg._lib
    sizes = {"dbsde_problem": L.Problem, "dbsde_config": L.Config, "dbsde_batch": L.Batch,
             "dbsde_outputs": L.Outputs, "dbsde_optim": L.Optim}
    for cname, ct in sizes.items():
        assert int(got[cname]) == ctypes.sizeof(ct), cname
    offs = {"dbsde_config.problem": L.Config.problem, "dbsde_config.T": L.Config.T,
            "dbsde_config.device": L.Config.device, "dbsde_batch.seed": L.Batch.seed,
            "dbsde_batch.path0": L.Batch.path0, "dbsde_batch.Xi": L.Batch.Xi,
            "dbsde_batch.xi_rows": L.Batch.xi_rows, "dbsde_optim.max_norm": L.Optim.max_norm,
            "dbsde_optim.step": L.Optim.step, "dbsde_problem.q3": L.Problem.q3,
            "dbsde_problem.kind": L.Problem.kind, "dbsde_problem.g_cols": L.Problem.g_cols,
            "dbsde_problem.u_clamp": L.Problem.u_clamp, "dbsde_problem.h_rho": L.Problem.h_rho,
            "dbsde_optim.alpha": L.Optim.alpha, "dbsde_optim.asgd_mu": L.Optim.asgd_mu,
            "dbsde_optim.loss": L.Optim.loss, "dbsde_optim.step_state": L.Optim.step_state,
            "dbsde_optim.step_parity": L.Optim.step_parity}
    for k, field in offs.items():
        assert int(got[k]) == field.offset, k


def test_evaluator_entry_points_validate_before_any_hip_call(lib):
    """dbsde_exact / dbsde_hjb_mc reject bad arguments with EINVAL (no GPU here)."""
    pkg = load_pkg()
    assert lib.dbsde_exact(9, None, None, 1, 1, 1.0, None, None, None, None) == pkg._lib.DBSDE_EINVAL
    assert lib.dbsde_hjb_mc(None, None, 1, 1, 1.0, 10, 0, None, None) == pkg._lib.DBSDE_EINVAL
    assert lib.dbsde_brownian_dim(None) == -1


def test_problem_kind_validation(lib):
    """Unknown problem kinds / terminal conditions and an odd Heston state are EINVAL."""
    pkg = load_pkg()
    cfg = pkg._lib.Config()
    for k, v in enumerate([6, 16, 16, 16, 16, 1]):
        cfg.layers[k] = v
    cfg.mode, cfg.activation, cfg.n_layers = 3, 0, 6
    ctx = ctypes.c_void_p()
    cfg.problem.kind = 7
    assert lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx)) == pkg._lib.DBSDE_EINVAL
    cfg.problem.kind, cfg.problem.g_kind = 0, 9
    assert lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx)) == pkg._lib.DBSDE_EINVAL
    cfg.problem.kind, cfg.problem.g_kind = 1, 2                 # Heston with an odd state dimension (5)
    assert lib.dbsde_create(ctypes.byref(cfg), ctypes.byref(ctx)) == pkg._lib.DBSDE_EINVAL
    assert b"even" in lib.dbsde_last_error(None)
