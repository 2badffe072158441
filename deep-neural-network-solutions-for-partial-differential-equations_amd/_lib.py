"""ctypes binding of include/dbsde.h (the C ABI of the HIP library).

The library is built in-tree by __graft_entry__.build() / build_lib.py into
lib/libdbsde.so.  There is no fallback: if the library (or a GPU) is missing,
every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("DBSDE_LIB") or os.path.join(LIB_DIR, "libdbsde.so")  # DBSDE_LIB: A/B experiments only

DBSDE_OK, DBSDE_EINVAL, DBSDE_EHIP, DBSDE_ENOMEM = 0, -1, -2, -3

MODES = {"FC": 0, "NAIS-Net": 1, "Resnet": 2, "Naisnet": 3}
ACTIVATIONS = {"Sine": 0, "ReLU": 1, "Tanh": 2}
G_KINDS = {"sumsq": 0, "call_sum": 1, "call_mean": 2, "log": 3, "smooth_call": 4}
PROBLEM_KINDS = {"diag": 0, "heston": 1}
OPTIMIZERS = {"Adam": 0, "AdamW": 1, "SGD": 2, "RMSprop": 3, "Adagrad": 4, "Adamax": 5, "Adadelta": 6, "ASGD": 7}
EXACT_KINDS = {"bsb": 0, "bs_call": 1, "basket_avg": 2, "basket_mean": 3}
ABI_VERSION = 3

# every symbol include/dbsde.h declares (checked by the CPU test suite)
EXPORTED = [
    "dbsde_abi_version", "dbsde_create", "dbsde_destroy", "dbsde_last_error", "dbsde_set_stream",
    "dbsde_param_count", "dbsde_param_used_mask", "dbsde_matrix_form", "dbsde_brownian_dim", "dbsde_set_corr", "dbsde_brownian", "dbsde_prefetch",
    "dbsde_prefetch_cancel",
    "dbsde_loss_grad", "dbsde_net_u", "dbsde_net_u_vjp", "dbsde_optimizer_step", "dbsde_exact", "dbsde_hjb_mc",
    "dbsde_profile_enable", "dbsde_profile_count", "dbsde_profile_read", "dbsde_profile_reset",
    "dbsde_vec_reduce", "dbsde_vec_axpby", "dbsde_lbfgs_direction", "dbsde_train_step",
    "dbsde_stream_order_by_events",
]
VEC_OPS = {"dot": 0, "asum": 1, "amax": 2}


class Problem(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("mu_a", ctypes.c_float), ("sig_a", ctypes.c_float),
                ("sig_b", ctypes.c_float), ("phi_r", ctypes.c_float), ("phi_c", ctypes.c_float),
                ("phi_zz", ctypes.c_float), ("g_kind", ctypes.c_int), ("strike", ctypes.c_float),
                ("q3", ctypes.c_int), ("g_cols", ctypes.c_int), ("g_alpha", ctypes.c_float),
                ("u_clamp", ctypes.c_int), ("h_kappa", ctypes.c_float), ("h_theta", ctypes.c_float),
                ("h_sigma", ctypes.c_float), ("h_rho", ctypes.c_float)]


class Config(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("activation", ctypes.c_int), ("n_layers", ctypes.c_int),
                ("layers", ctypes.c_int * 16), ("problem", Problem), ("T", ctypes.c_float),
                ("device", ctypes.c_int)]


class Batch(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int), ("N", ctypes.c_int), ("t", ctypes.c_void_p), ("W", ctypes.c_void_p),
                ("seed", ctypes.c_ulonglong), ("offset", ctypes.c_ulonglong), ("path0", ctypes.c_longlong),
                ("Xi", ctypes.c_void_p),
                ("xi_rows", ctypes.c_int)]


class Outputs(ctypes.Structure):
    _fields_ = [("loss", ctypes.c_void_p), ("X", ctypes.c_void_p), ("Y", ctypes.c_void_p),
                ("Z", ctypes.c_void_p)]


class Optim(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("max_norm", ctypes.c_float), ("step", ctypes.c_longlong), ("alpha", ctypes.c_float),
                ("rho", ctypes.c_float), ("lr_decay", ctypes.c_float), ("lambd", ctypes.c_float),
                ("asgd_eta", ctypes.c_float), ("asgd_mu", ctypes.c_float), ("loss", ctypes.c_void_p),
                ("step_state", ctypes.c_void_p), ("step_parity", ctypes.c_int)]


_LIB = None


def load():
    """Load lib/libdbsde.so (no HIP call is made by loading)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build the HIP library first (python __graft_entry__.py build)")
    lib = ctypes.CDLL(LIB_PATH)
    vp, i, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
    sig = {
        "dbsde_abi_version": (i, []),
        "dbsde_create": (i, [ctypes.POINTER(Config), ctypes.POINTER(vp)]),
        "dbsde_destroy": (None, [vp]),
        "dbsde_last_error": (ctypes.c_char_p, [vp]),
        "dbsde_set_stream": (i, [vp, vp]),
        "dbsde_stream_order_by_events": (i, [ctypes.POINTER(ctypes.c_char_p)]),
        "dbsde_param_count": (ll, [vp]),
        "dbsde_param_used_mask": (i, [vp, vp, ll]),
        "dbsde_matrix_form": (i, [vp]),
        "dbsde_brownian_dim": (i, [vp]),
        "dbsde_set_corr": (i, [vp, vp, i]),
        "dbsde_brownian": (i, [vp, ctypes.POINTER(Batch), vp, vp, i]),
        "dbsde_prefetch": (i, [vp, ctypes.POINTER(Batch)]),
        "dbsde_prefetch_cancel": (i, [vp]),
        "dbsde_exact": (i, [i, vp, vp, ll, i, ctypes.c_float, vp, vp, vp, vp]),
        "dbsde_hjb_mc": (i, [vp, vp, i, i, ctypes.c_float, ll, ctypes.c_ulonglong, vp, vp]),
        "dbsde_loss_grad": (i, [vp, vp, ctypes.POINTER(Batch), vp, ctypes.POINTER(Outputs)]),
        "dbsde_net_u": (i, [vp, vp, i, vp, vp, vp, vp]),
        "dbsde_net_u_vjp": (i, [vp, vp, i, vp, vp, vp, vp, vp]),
        "dbsde_optimizer_step": (i, [vp, vp, vp, vp, vp, ctypes.POINTER(Optim)]),
        "dbsde_profile_enable": (i, [vp, i]),
        "dbsde_profile_count": (i, [vp]),
        "dbsde_profile_read": (i, [vp, i, ctypes.c_char_p, i, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ll)]),
        "dbsde_profile_reset": (i, [vp]),
        "dbsde_train_step": (i, [vp, vp, ctypes.POINTER(Batch), vp, vp, vp, ctypes.POINTER(Optim),
                                 ctypes.POINTER(Outputs)]),
        "dbsde_vec_reduce": (i, [vp, i, vp, vp, ll, ctypes.POINTER(ctypes.c_double)]),
        "dbsde_vec_axpby": (i, [vp, vp, vp, vp, ll, ctypes.c_float, ctypes.c_float]),
        "dbsde_lbfgs_direction": (i, [vp, vp, vp, vp, ll, ll, vp, vp, i, ctypes.c_float, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.dbsde_abi_version() != ABI_VERSION:
        raise RuntimeError("libdbsde ABI version mismatch")
    _LIB = lib
    return lib


def check(rc, ctx=None):
    """Map a C status to the reference's Python exception types."""
    if rc == DBSDE_OK:
        return
    msg = load().dbsde_last_error(ctx)
    msg = msg.decode() if msg else "unknown error"
    if rc == DBSDE_EINVAL:
        raise ValueError(msg)
    if rc == DBSDE_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)
